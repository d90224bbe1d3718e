"""Diagnostic: one IK handle on its own stream while other streams run
unrelated torch work (GEMMs / copies). Its poses must equal the serial run.
    python scripts/diag_perturb.py MODE REPS [B]   MODE in gemm, copy, ik2"""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from temporal_inverse_kinematics_amd import synthetic as syn
from temporal_inverse_kinematics_amd.inference import synthetic_model

MODE = sys.argv[1] if len(sys.argv) > 1 else "gemm"
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
T = 64
dev = torch.device("cuda:0")
x = torch.from_numpy(syn.synthetic_windows(B, T, seed=0)).to(dev)
with torch.no_grad():
    m = synthetic_model(win_size=T, device=dev).regressor
    ref = m(x)["poses"].clone()
    torch.cuda.synchronize()
    s_ik = torch.cuda.Stream()
    others = [torch.cuda.Stream() for _ in range(3)]
    a = torch.randn(4096, 4096, device=dev)
    bufs = [torch.empty(64 << 20, device=dev) for _ in range(6)]
    diffs = []
    for rep in range(REPS):
        ev = torch.cuda.Event(); ev.record()
        for k, s in enumerate(others):
            with torch.cuda.stream(s):
                s.wait_event(ev)
                for _ in range(6):
                    if MODE == "gemm":
                        a @ a
                    else:
                        bufs[2 * k].copy_(bufs[2 * k + 1])
        with torch.cuda.stream(s_ik):
            s_ik.wait_event(ev)
            outs = [m(x)["poses"] for _ in range(4)]
        torch.cuda.synchronize()
        diffs.append(max(float((o - ref).abs().max()) for o in outs))
print(json.dumps({"mode": MODE, "B": B, "env": {k: v for k, v in os.environ.items() if k.startswith("TIK_")},
                  "max_diff_per_rep": diffs}))
