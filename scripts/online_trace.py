"""Per-phase timing of the online-IK dataflow kernel (TIK_ONLINE_TRACE=1).

    python scripts/online_trace.py [--win 64] [--pushes 60]

Prints, per phase, when its tasks took their tickets, when their inputs were
staged (every element carried the launch's tag) and when they finished,
relative to the step's first ticket (us)."""
import argparse, ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TIK_ONLINE_TRACE"] = "1"
import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--win", type=int, default=64)
    ap.add_argument("--pushes", type=int, default=60)
    a = ap.parse_args()
    from temporal_inverse_kinematics_amd import _build, _lib, synthetic as syn
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    _build.build()
    m = synthetic_model(win_size=a.win, device="cuda")
    s = OnlineIK(m, use_graph=True)
    seq = syn.load_sample_coco()
    for i in range(a.pushes):
        s.push(seq[i % seq.shape[0]])
    lib = _lib.load()
    n = lib.tik_debug_stream_trace(s._s, None, 0)
    buf = (ctypes.c_longlong * (8 * n))()
    lib.tik_debug_stream_trace(s._s, buf, 8 * n)
    tr = np.frombuffer(buf, dtype=np.int64).reshape(n, 8).astype(np.float64)
    t0 = tr[:, 0].min()
    us = (tr[:, :7] - t0) / 100.0   # 100 MHz ticks -> us
    # phase table (stream.cpp setup_online)
    strides = [1, 1, 2, 1, 1, 2, 2, 2]
    couts = [64, 64, 128, 128, 128, 128, 256, 256]
    W = 2 * (a.win // 2) + 1
    tin, t = [], W
    for st in strides:
        tin.append(t)
        t = (t - 1) // st + 1
    nin, nout, need = [0] * 8, [0] * 8, 1
    for l in range(7, -1, -1):
        nout[l] = need
        nin[l] = min(tin[l], strides[l] * (need - 1) + 2)
        need = nin[l]
    phases = []
    for l in range(8):
        phases += [(f"G{l}", nin[l] * couts[l] // 16), (f"T{l}", nout[l] * couts[l] // 16)]
    phases += [("H", 512 // 16)]
    assert sum(c for _, c in phases) == n, (n, phases)
    k = 0
    print(f"{n} tasks, {len(set(tr[:, 7].astype(int)))} workgroups; step span {us[:, 6].max():.1f} us")
    print(f"{'phase':6s} {'tasks':>5s} {'grab':>14s} {'staged':>14s} {'done':>14s} {'run(staged->done)':>18s}")
    for name, c in phases:
        g, q, r, d = us[k:k + c, 0], us[k:k + c, 1], us[k:k + c, 2], us[k:k + c, 6]
        extra = ""
        if name[0] in "GT":
            cp, rd, sd = us[k:k + c, 3], us[k:k + c, 4], us[k:k + c, 5]
            extra = (f"  | wait+load {np.mean(r - q):4.2f} compute {np.mean(cp - r):4.2f} reduce {np.mean(rd - cp):4.2f}"
                     f" epi+store {np.mean(sd - rd):4.2f} end {np.mean(d - sd):4.2f}")
        print(f"{name:6s} {c:5d} {g.min():6.1f}-{g.max():6.1f} {r.min():6.1f}-{r.max():6.1f} {d.min():6.1f}-{d.max():6.1f}"
              f"   mean {np.mean(d - r):5.2f} max {np.max(d - r):5.2f}{extra}")
        k += c


if __name__ == "__main__":
    main()
