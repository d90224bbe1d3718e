"""Diagnostic: P processes on the same GPU, each running the IK forward of
its own handle repeatedly; each checks every repetition against its first."""
import sys, os, json, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    from temporal_inverse_kinematics_amd import synthetic as syn
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    dev = torch.device("cuda:0")
    x = torch.from_numpy(syn.synthetic_windows(256, 64, seed=0)).to(dev)
    with torch.no_grad():
        m = synthetic_model(win_size=64, device=dev).regressor
        ref = m(x)["poses"].clone()
        worst = 0.0
        import time
        secs = float(os.environ.get("AGG_SECONDS", "0"))
        t0, it = time.time(), 0
        while (it < 300) if secs <= 0 else (time.time() - t0 < secs):
            worst = max(worst, float((m(x)["poses"] - ref).abs().max()))
            it += 1
    print(worst)
    sys.exit(0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
procs = [subprocess.Popen([sys.executable, __file__, "child"], stdout=subprocess.PIPE, text=True) for _ in range(P)]
outs = [p.communicate(timeout=200)[0].strip() for p in procs]
print(json.dumps({"P": P, "worst_per_process": outs}))
