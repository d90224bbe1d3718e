"""Diagnostic (TIK_CHECKSUM): P processes run the IK forward concurrently;
each compares the per-launch output checksums of every repetition with its
first run and tallies the FIRST launch whose output differs."""
import sys, os, json, subprocess, ctypes, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    os.environ["TIK_CHECKSUM"] = "1"
    import torch
    from temporal_inverse_kinematics_amd import _lib, synthetic as syn
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    lib = _lib.load()
    buf = ctypes.create_string_buffer(1 << 16)
    dev = torch.device("cuda:0")
    x = torch.from_numpy(syn.synthetic_windows(256, 64, seed=0)).to(dev)
    def run():
        lib.tik_debug_checksums(buf, len(buf))
        m(x)
        lib.tik_debug_checksums(buf, len(buf))
        return [kv.split(":") for kv in buf.value.decode().strip(";").split(";")]
    with torch.no_grad():
        m = synthetic_model(win_size=64, device=dev).regressor
        ref = run()
        first_bad, nrep, t0 = {}, 0, time.time()
        while time.time() - t0 < float(sys.argv[2]):
            cur = run()
            nrep += 1
            for (la, a), (lb, b) in zip(ref, cur):
                if a != b:
                    first_bad[la] = first_bad.get(la, 0) + 1
                    break
    print(json.dumps({"reps": nrep, "launches": [l for l, _ in ref], "first_bad": first_bad}))
    sys.exit(0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
procs = [subprocess.Popen([sys.executable, __file__, "child", "40"], stdout=subprocess.PIPE, text=True) for _ in range(P)]
for p in procs:
    print(p.communicate(timeout=200)[0].strip())
