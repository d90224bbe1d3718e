"""SURVEY.md §8f row 4 (optimizer half): the IKPoseTrainer training step on the GPU.

    python bench_train.py [--batch 256] [--T 9] [--steps 50] [--warmup 5]

Workload: the reference's training defaults (pose_trainer.py:204-230:
--bs 256 windows, --win_size 9 -> 9-frame windows, 1 output frame, Adam lr
1e-4), synthetic AMASS-shaped windows and targets resident on the device,
seeded synthetic weights. One step = train-mode forward + MSE + backward +
Adam (GpuTrainer.step -> tik_trainer_step), device dropout masks. Metric:
training windows/s. Algorithmic work per window: forward FLOPs of the
dense contractions (oracle count, 92.9 MFLOP at T=9) x 3 (forward, input
gradient, weight gradient). CPU baseline: oracle/train.py (the reference's
step restated in PyTorch fp32 autograd) on the host, a bounded sample.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def fwd_flops_per_window(T, layers=((3, 64, 1), (64, 64, 1), (64, 128, 2), (128, 128, 1), (128, 128, 1),
                                    (128, 128, 2), (128, 256, 2), (256, 256, 2))):
    V, fl, t = 17, 0.0, T
    for cin, cout, s in layers:
        to = (t - 1) // s + 1
        fl += 2.0 * t * V * cin * cout + 2.0 * t * V * V * cout + 2.0 * to * V * 3 * cout * cout
        if not (cin == cout and s == 1):
            fl += 2.0 * to * V * cin * cout
        t = to
    fl += 2.0 * t * (V * 256 * 512 + 512 * 66)
    return fl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--T", type=int, default=9)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from temporal_inverse_kinematics_amd import _build, synthetic as syn
    from temporal_inverse_kinematics_amd.models import IKPoseTrainer, default_hparams
    from temporal_inverse_kinematics_amd.trainer import GpuTrainer
    _build.build()
    m = IKPoseTrainer(default_hparams(win_size=a.T))
    sd = syn.ik_state_dict(m.regressor.backbone.graph.A, seed=0)
    own = m.regressor.state_dict()
    m.regressor.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items() if k in own}, strict=False)
    tr = GpuTrainer(m, lr=1e-4)
    B, T = a.batch, a.T
    Tp = T
    for s in m.regressor.backbone.strides:
        Tp = (Tp - 1) // s + 1
    xs = [torch.from_numpy(syn.synthetic_windows(B, T, seed=50 + i)).cuda() for i in range(4)]
    rng = np.random.default_rng(0)
    ys = [torch.from_numpy(rng.normal(0, 0.5, (B, Tp, 66)).astype(np.float32)).cuda() for _ in range(4)]
    for i in range(a.warmup):
        tr.step(xs[i % 4], ys[i % 4], seed=i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = tr.step(xs[i % 4], ys[i % 4], seed=1000 + i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    fl = 3.0 * fwd_flops_per_window(T)
    out = {"metric": "IK training windows/sec (train-mode forward + MSE + backward + Adam)",
           "value": round(B / dt, 1), "unit": "windows/s", "ms_per_step": round(dt * 1e3, 4),
           "higher_is_better": True, "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "dtype": "f32",
           "data": "synthetic (AMASS-shaped windows, random target poses, seeded synthetic weights)",
           "config": {"workload": f"IKPoseTrainer step, bs={B} x {T}-frame windows -> {Tp} output frame(s), Adam lr 1e-4",
                      "batch": B, "window_frames": T},
           "algorithmic_tflops": round(fl * B / dt / 1e12, 2), "mflop_per_window": round(fl / 1e6, 2),
           "roofline": {"scope": "whole step (forward + backward GEMM FLOPs / step time)", "bound": "mfma",
                        "achieved": round(fl * B / dt / 1e12, 2), "peak": 157.3, "unit": "TFLOP/s",
                        "frac": round(fl * B / dt / 1e12 / 157.3, 4),
                        "peak_basis": "dense fp32 MFMA (v_mfma_f32_16x16x4_f32), MI355X_MICROARCH.md"},
           "loss_last": float(loss)}
    if not a.no_cpu_baseline:
        from oracle import train as otr
        nb = 16
        x = syn.synthetic_windows(nb, T, seed=9)
        tgt = np.random.default_rng(1).normal(0, 0.5, (nb, Tp, 66)).astype(np.float32)
        mask = (np.random.default_rng(2).random((nb * Tp, 512)) < 0.3).astype(np.float32)
        otr.train_steps(sd, [(x, tgt, mask)])
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < a.cpu_seconds:
            otr.train_steps(sd, [(x, tgt, mask)])
            done += nb
        d = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(done / d, 1), "unit": "windows/s", "cores": torch.get_num_threads(),
                               "kind": "port", "sample": f"{done} windows in steps of {nb} through oracle/train.py "
                                                         f"(PyTorch fp32 autograd on the host) in {d:.1f}s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
