"""Config #4: SMPL-X full 55-joint FK + 10475-vertex LBS, batch=4096, 1 GPU.

    python bench_fk.py [--batch 4096] [--steps 10] [--warmup 20]

Prints one JSON line: bodies/s, and per kernel (HIP events around every launch
of a second pass of the same steps, tik_fk_profile) the algorithmic TFLOP/s of
the blend-shape and skinning GEMMs against the bf16x3 MFMA roof and the
vertex bytes over HBM; then the oracle CPU baseline. bench.py reuses
measure_fk() for its "fk" key.
"""
import argparse, ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BF16_MFMA_PEAK_TFLOPS = 2516.6   # dense bf16 MFMA (MI355X_MICROARCH.md); bf16x3 runs 6 products per fp32 product
HBM_PEAK_GBS = 8000.0
DTYPES = {"bf16x3": "f32 via bf16x3 (3 bf16 planes, 6 MFMA products, fp32 accumulate; fp32 exponent range)",
          "fp32": "f32 (exact fp32 MFMA)"}


def measure_fk(batch=4096, steps=10, warmup=20):
    """Time `steps` FK+LBS forwards of `batch` bodies (inputs resident), then the
    same steps again with per-launch HIP events: the step time and the per-kernel
    roofline of the two LBS GEMMs (bf16x3: 6 bf16 MFMA products per fp32 product)."""
    import torch
    from temporal_inverse_kinematics_amd import _build, _lib, synthetic as syn
    from temporal_inverse_kinematics_amd.smplx_fk import SMPLX
    _build.build()
    c = syn.synthetic_smplx_constants(seed=1)
    m = SMPLX(c, batch_size=batch)
    pose, betas = syn.synthetic_fk_inputs(batch, seed=1)
    P, Bt = torch.from_numpy(pose).cuda(), torch.from_numpy(betas).cuda()
    # outputs into preallocated buffers (a serving loop's); 20 warmup steps: the
    # first ~10 FK steps on a fresh box run 5-20 % slow (clocks / caches settling,
    # scripts/diag_fkgap.py: 1.16 -> 0.98 ms/step)
    out = (torch.empty((batch, m.num_joints, 3), device="cuda"), torch.empty((batch, m.num_verts, 3), device="cuda"))
    for _ in range(warmup):
        m.full_forward(P, Bt, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        m.full_forward(P, Bt, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    lib = _lib.load()
    _lib.check(lib.tik_fk_profile(m._h, 8 * steps))
    for _ in range(steps):
        m.full_forward(P, Bt, out=out)
    torch.cuda.synchronize()
    agg = {}
    lab = ctypes.create_string_buffer(64)
    kms, fl, by = ctypes.c_float(), ctypes.c_double(), ctypes.c_double()
    for i in range(_lib.check(lib.tik_fk_profile_count(m._h))):
        _lib.check(lib.tik_fk_profile_read(m._h, i, lab, 64, ctypes.byref(kms), ctypes.byref(fl), ctypes.byref(by)))
        a = agg.setdefault(lab.value.decode(), [0.0, 0, 0.0, 0.0])
        a[0] += kms.value; a[1] += 1; a[2] += fl.value; a[3] += by.value
    lib.tik_fk_profile(m._h, 0)
    nprod = 6 if m.precision == "bf16x3" else 1
    roof = BF16_MFMA_PEAK_TFLOPS / 6 if nprod == 6 else 157.3
    kernels = {}
    for k, (t, n, f, b) in agg.items():
        s = t / 1e3
        d = {"avg_ms": round(t / n, 4), "share": round(t / sum(v[0] for v in agg.values()), 3)}
        if f > 0:
            d.update({"tflops": round(f / s / 1e12, 2), "mfma_frac": round(f / s / 1e12 / roof, 4)})
        d.update({"gbs": round(b / s / 1e9, 1), "hbm_frac": round(b / s / 1e9 / HBM_PEAK_GBS, 4)})
        kernels[k] = d
    V = c["v_template"].shape[0]
    gemm_flops = 2.0 * batch * 3 * V * 507 + 2.0 * batch * V * 12 * 55 + 18.0 * batch * V
    vert_bytes = batch * V * 3 * 4
    return {"metric": "SMPL-X FK+LBS bodies/sec", "value": round(batch / (ms / 1e3), 1), "unit": "bodies/s",
            "n_gpus": 1, "ms_per_step": round(ms, 4), "steps": steps, "warmup": warmup,
            "dtype": DTYPES.get(m.precision, m.precision),
            "config": {"workload": f"SMPL-X 55-joint FK + {V}-vertex LBS + 144 joints, batch={batch}"},
            "gemm_tflops": round(gemm_flops / (ms / 1e3) / 1e12, 2), "mflop_per_body": round(gemm_flops / batch / 1e6, 2),
            "mfma_roof_tflops": round(roof, 1),
            "vertex_gbs": round(vert_bytes / (ms / 1e3) / 1e9, 1),
            "vertex_hbm_frac": round(vert_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "bytes_out_per_body": (V * 3 + 144 * 3) * 4, "kernels": kernels,
            "outputs": "joints and vertices written into preallocated buffers (SMPLX.full_forward(out=...))",
            "basis": "kernels: HIP events around each launch of a second pass of the same steps (tik_fk_profile); "
                     "tflops = algorithmic fp32 FLOPs / event time, mfma_frac against the bf16x3 roof "
                     f"({BF16_MFMA_PEAK_TFLOPS} TF dense bf16 / 6 products); vertex_gbs = vertex bytes written / step time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()
    from temporal_inverse_kinematics_amd import synthetic as syn
    out = measure_fk(a.batch, a.steps, a.warmup)
    from oracle import smplx_lbs as sl
    c = syn.synthetic_smplx_constants(seed=1)
    pose, betas = syn.synthetic_fk_inputs(16, seed=1)
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < a.cpu_seconds:
        sl.smplx_forward(c, pose, betas); n += 16
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": round(n / dt, 1), "unit": "bodies/s", "kind": "port",
                           "sample": f"{n} bodies through oracle/smplx_lbs.py (numpy f64) in {dt:.1f}s"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
