"""Experiment: the 1024-window forward as S concurrent sub-batches on S HIP
streams (one model handle each) vs one launch sequence on one stream."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from temporal_inverse_kinematics_amd import synthetic as syn
from temporal_inverse_kinematics_amd.inference import synthetic_model


def run(S, B=1024, T=64, steps=30):
    dev = torch.device("cuda:0")
    models = [synthetic_model(win_size=T, device=dev).regressor for _ in range(S)]
    x = torch.from_numpy(syn.synthetic_windows(B, T, seed=0)).to(dev)
    parts = list(x.chunk(S))
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [None] * S

    def step():
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event(); ev.record(cur)
        for i in range(S):
            with torch.cuda.stream(streams[i]):
                streams[i].wait_event(ev)
                outs[i] = models[i](parts[i])["poses"]
        for i in range(S):
            cur.wait_stream(streams[i])
    with torch.no_grad():
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    y = torch.cat(outs)
    return dt, y


if __name__ == "__main__":
    base, y1 = run(1)
    res = {"S1_ms": base * 1e3, "S1_fps": 1024 / base}
    for S in (2, 4):
        dt, y = run(S)
        res[f"S{S}_ms"] = dt * 1e3
        res[f"S{S}_fps"] = 1024 / dt
        res[f"S{S}_maxdiff"] = float((y - y1).abs().max())
    print(json.dumps(res))
