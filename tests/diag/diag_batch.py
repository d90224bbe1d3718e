"""Diagnostic: the IK forward of a window must not depend on the batch it is
in. Runs the 1024-window batch whole and as sub-batches of several sizes
(one handle; then S handles on S streams) and reports max |difference|; the
worst window is checked against the CPU oracle."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from temporal_inverse_kinematics_amd import synthetic as syn
from temporal_inverse_kinematics_amd.inference import synthetic_model

dev = torch.device("cuda:0")
B, T = 1024, 64
xn = syn.synthetic_windows(B, T, seed=0)
x = torch.from_numpy(xn).to(dev)
res = {}
with torch.no_grad():
    m = synthetic_model(win_size=T, device=dev).regressor
    y = m(x)["poses"].clone()
    for n in (512, 256, 128, 100, 333, 64):
        parts = [m(c)["poses"] for c in x.split(n)]
        d = (torch.cat(parts) - y).abs()
        res[f"one_handle_{n}"] = float(d.max())
        if float(d.max()) > 0:
            res[f"one_handle_{n}_worst_window"] = int(d.amax(dim=(1, 2)).argmax())
    torch.cuda.synchronize()
    for S in (2, 4):
        models = [synthetic_model(win_size=T, device=dev).regressor for _ in range(S)]
        streams = [torch.cuda.Stream() for _ in range(S)]
        parts = list(x.chunk(S))
        for rep in range(3):
            outs = [None] * S
            ev = torch.cuda.Event(); ev.record()
            for i in range(S):
                with torch.cuda.stream(streams[i]):
                    streams[i].wait_event(ev)
                    outs[i] = models[i](parts[i])["poses"]
            for s in streams:
                torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            d = (torch.cat(outs) - y).abs()
            res[f"streams{S}_rep{rep}"] = float(d.max())
            if float(d.max()) > 0:
                res[f"streams{S}_rep{rep}_worst"] = int(d.amax(dim=(1, 2)).argmax())
        # same, serialised on the default stream
        outs = [models[i](parts[i])["poses"] for i in range(S)]
        res[f"serial{S}"] = float((torch.cat(outs) - y).abs().max())
    # oracle on a few windows (the worst ones, if any)
    from oracle import stgcn as orc
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    idx = sorted({v for k, v in res.items() if k.endswith("worst") or k.endswith("worst_window")} | {0, 1023})[:6]
    ref = orc.pose_regressor(xn[idx], sd)["poses"]
    res["oracle_windows"] = idx
    res["oracle_maxdiff_full"] = float(np.abs(y[idx].cpu().numpy() - ref).max())
print(json.dumps(res))
