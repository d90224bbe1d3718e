"""SURVEY.md §8f row 4 (data half): AmassDataset training-data generation on
the GPU (temporal_inverse_kinematics_amd/training_data.py).

    python bench_train_data.py [--seqs 64] [--frames 1000] [--batch 4096] [--steps 50]

Workload: synthetic AMASS-shaped sequences (156 pose columns, random betas,
three genders) on the seeded synthetic SMPL-X constants; window 64 (65
frames), Gaussian keypoint noise on. Two numbers: the per-epoch regeneration
(root rotation + SMPL-X FK joints of every frame, frames/s) and the item
batches (windows + targets, items/s, inputs resident on the device). CPU
baseline: oracle/amass.py's __getitem__ restatement on the same FK joints
(numpy, one host thread), a bounded sample."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=64)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from temporal_inverse_kinematics_amd import _build
    from temporal_inverse_kinematics_amd.smplx_fk import load_smplx_models
    from temporal_inverse_kinematics_amd.training_data import AmassDataset
    _build.build()
    rng = np.random.default_rng(0)
    seqs = []
    for i in range(a.seqs):
        t = np.linspace(0, 8 * np.pi, a.frames, dtype=np.float32)[:, None]
        poses = (rng.normal(0, 0.3, (1, 156)) + rng.normal(0, 0.2, (1, 156)) * np.sin(t + i)).astype(np.float32)
        seqs.append({"poses": poses, "betas": rng.normal(0, 1, 10).astype(np.float32),
                     "gender": ["male", "female", "neutral"][i % 3]})
    models = load_smplx_models(None, "cuda", batch_size=9)
    ds = AmassDataset(models, seqs, window_size=64, keypoint_format="coco", add_gaussian_noise=True)
    # per-epoch regeneration
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for e in range(reps):
        ds.on_epoch_end(e + 1)
    torch.cuda.synchronize()
    regen = (time.perf_counter() - t0) / reps
    n = len(ds)
    idx = [np.random.default_rng(s).integers(0, n, a.batch) for s in range(a.steps + 5)]
    for s in range(5):
        ds.get_batch(idx[s])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(a.steps):
        ds.get_batch(idx[5 + s])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    out = {"metric": "AmassDataset training items/s (window 64, noise)", "value": round(a.batch / dt, 1),
           "unit": "items/s", "ms_per_batch": round(dt * 1e3, 4), "batch": a.batch, "n_gpus": 1,
           "regen_frames_per_s": round(n / regen, 1), "regen_ms_per_epoch": round(regen * 1e3, 3),
           "dtype": "fp32 (FK: bf16x3 split MFMA, fp32 range)", "data": f"synthetic: {a.seqs} sequences x {a.frames} frames",
           "config": {"workload": "data_amass.AmassDataset: per-epoch root rotation + SMPL-X FK joints; "
                                  "items = COCO-17 window + noise + target pose"}}
    if not a.no_cpu_baseline:
        from oracle import amass as oa
        joints = [d["keypoints_3d"].cpu().numpy() for d in ds.data_anims]
        poses = [d["poses"].cpu().numpy() for d in ds.data_anims]
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 10.0:
            s = k % len(joints)
            oa.getitem(joints[s], poses[s], ds.data_anims[s]["betas"], 32 + k % (a.frames - 64), 32, k,
                       add_noise=True, seed=ds.noise_key)
            k += 1
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(k / el, 1), "unit": "items/s", "cores": 1, "kind": "port",
                               "sample": f"{k} items through oracle/amass.py getitem (numpy) in {el:.1f}s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
