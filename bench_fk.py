"""Config #4: SMPL-X full 55-joint FK + 10475-vertex LBS, batch=4096, 1 GPU.

    python bench_fk.py [--batch 4096] [--steps 10] [--warmup 3]

Prints one JSON line: bodies/s, per-kernel times (rocprof-comparable HIP
events are not needed here: the step is timed with torch.cuda events), the
MFMA roofline of the two LBS GEMMs, and the oracle CPU baseline.
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()
    import numpy as np, torch
    from temporal_inverse_kinematics_amd import _build, synthetic as syn
    from temporal_inverse_kinematics_amd.smplx_fk import SMPLX
    _build.build()
    c = syn.synthetic_smplx_constants(seed=1)
    m = SMPLX(c, batch_size=a.batch)
    pose, betas = syn.synthetic_fk_inputs(a.batch, seed=1)
    P, Bt = torch.from_numpy(pose).cuda(), torch.from_numpy(betas).cuda()
    for _ in range(a.warmup):
        m.full_forward(P, Bt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        m.full_forward(P, Bt)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    V, B = c["v_template"].shape[0], a.batch
    gemm_flops = 2.0 * B * 3 * V * 507 + 2.0 * B * V * 12 * 55 + 18.0 * B * V
    out = {"metric": "SMPL-X FK+LBS bodies/sec", "value": round(B / (ms / 1e3), 1), "unit": "bodies/s",
           "n_gpus": 1, "ms_per_step": round(ms, 4),
           "dtype": {"bf16x3": "f32 via bf16x3 (3 bf16 planes, 6 MFMA products, fp32 accumulate; fp32 exponent range)",
                     "f16x3": "f32 via f16x3 (3 MFMA products; f16 range, narrower than fp32)",
                     "fp32": "f32 (exact fp32 MFMA)"}.get(m.precision, m.precision), "config": {"workload": f"SMPL-X 55-joint FK + {V}-vertex LBS + 144 joints, batch={B}"},
           "gemm_tflops": round(gemm_flops / (ms / 1e3) / 1e12, 2), "mflop_per_body": round(gemm_flops / B / 1e6, 2),
           "bytes_out_per_body": (V * 3 + 144 * 3) * 4}
    from oracle import smplx_lbs as sl
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < a.cpu_seconds:
        sl.smplx_forward(c, pose[:16], betas[:16]); n += 16
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": round(n / dt, 1), "unit": "bodies/s", "kind": "port",
                           "sample": f"{n} bodies through oracle/smplx_lbs.py (numpy f64) in {dt:.1f}s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
