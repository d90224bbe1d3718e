"""Config #5: streaming sliding-window (stride 1) online IK, hipGraph-captured
step, per-frame latency (push of one frame -> its solved pose on the host).

    python bench_stream.py [--frames 10000] [--warmup 100] [--win 64]
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--win", type=int, default=64)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--precision", default="f16x3", choices=["f16x3", "fp32"])
    a = ap.parse_args()
    import numpy as np
    from temporal_inverse_kinematics_amd import _build, synthetic as syn
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    _build.build()
    seq0 = syn.load_sample_coco()
    reps = -(-a.frames // seq0.shape[0])
    rng = np.random.default_rng(0)
    seq = np.concatenate([seq0 + rng.normal(0, 0.01, seq0.shape).astype(np.float32) for _ in range(reps)])[:a.frames]
    m = synthetic_model(win_size=a.win, device="cuda", precision=a.precision)
    s = OnlineIK(m, use_graph=not a.no_graph)
    for i in range(a.warmup):
        s.push(seq[i % seq.shape[0]])
    s.reset()
    lat = np.empty(a.frames)
    for i in range(a.frames):
        t0 = time.perf_counter()
        s.push(seq[i])
        lat[i] = time.perf_counter() - t0
    lat_us = lat * 1e6
    out = {"metric": "online IK per-frame latency (p50)", "value": round(float(np.percentile(lat_us, 50)), 2),
           "unit": "us", "higher_is_better": False, "p99_us": round(float(np.percentile(lat_us, 99)), 2),
           "mean_us": round(float(lat_us.mean()), 2), "frames_per_s": round(a.frames / lat.sum(), 1),
           "n_gpus": 1, "dtype": "fp32" if s.path == "dataflow" else a.precision, "step": s.path,
           "config": {"workload": f"stride-1 sliding window, win_size={a.win} (T={2 * (a.win // 2) + 1}), B=1, "
                                  f"{'hipGraph replay' if not a.no_graph else 'eager launches'} per frame"
                                  + (" (one dataflow kernel, only the frames pose row 0 depends on)"
                                     if s.path == "dataflow" else " (layered forward on the whole window)"),
                      "frames": a.frames, "warmup": a.warmup}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
