"""Config #5: streaming sliding-window (stride 1) online IK, hipGraph-captured
step, per-frame latency (push of one frame -> its solved pose on the host).

    python bench_stream.py [--frames 10000] [--warmup 100] [--win 64]

bench.py reuses measure_online() for its "online" key.
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def measure_online(frames=10000, warmup=100, win=64, use_graph=True, precision="bf16x3"):
    """Push `frames` frames of the sample sequence (noised repeats) one at a
    time through OnlineIK and time each push (frame in -> pose on the host)."""
    import numpy as np
    from temporal_inverse_kinematics_amd import _build, synthetic as syn
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    from temporal_inverse_kinematics_amd.streaming import OnlineIK
    _build.build()
    seq0 = syn.load_sample_coco()
    reps = -(-frames // seq0.shape[0])
    rng = np.random.default_rng(0)
    seq = np.concatenate([seq0 + rng.normal(0, 0.01, seq0.shape).astype(np.float32) for _ in range(reps)])[:frames]
    m = synthetic_model(win_size=win, device="cuda", precision=precision)
    s = OnlineIK(m, use_graph=use_graph)
    for i in range(warmup):
        s.push(seq[i % seq.shape[0]])
    s.reset()
    lat = np.empty(frames)
    for i in range(frames):
        t0 = time.perf_counter()
        s.push(seq[i])
        lat[i] = time.perf_counter() - t0
    lat_us = lat * 1e6
    return {"metric": "online IK per-frame latency (p50)", "value": round(float(np.percentile(lat_us, 50)), 2),
            "unit": "us", "higher_is_better": False, "p99_us": round(float(np.percentile(lat_us, 99)), 2),
            "mean_us": round(float(lat_us.mean()), 2), "frames_per_s": round(frames / lat.sum(), 1),
            "n_gpus": 1, "dtype": ("f32: gcn and temporal convs via bf16x3 MFMA (3 bf16 planes, 6 products, fp32 accumulate), "
                                             "joint 16, graph mix and head in fp32 FMAs") if s.path == "dataflow" else precision, "step": s.path,
            "config": {"workload": f"stride-1 sliding window, win_size={win} (T={2 * (win // 2) + 1}), B=1, "
                                   f"{'hipGraph replay' if use_graph else 'eager launches'} per frame"
                                   + (" (one dataflow kernel, only the frames pose row 0 depends on)"
                                      if s.path == "dataflow" else " (layered forward on the whole window)"),
                       "frames": frames, "warmup": warmup}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--win", type=int, default=64)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "fp32"])
    a = ap.parse_args()
    print(json.dumps(measure_online(a.frames, a.warmup, a.win, not a.no_graph, a.precision)))


if __name__ == "__main__":
    main()
