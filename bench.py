"""Headline benchmark: IK frames/s (COCO-17 -> SMPL-X body pose) on MI355X.

One step = one fused IK forward of the rank's batch of B=1024 synthetic
AMASS-shaped windows (T=64, inputs already resident in HBM), and for N>1 the
RCCL all-gather of the (B,T',66) pose parameters to every rank over xGMI
(BASELINE.json config #2 at N=1, config #3 = 8x1024 at N=8; weak scaling).
IK frame := one window -> one solved frame (inference.py:58-64).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--T T]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line with the metric, the roofline of the dominant
kernel (HIP events around its launches inside the timed region) and a CPU
baseline (the oracle, fixture-pinned to the reference, on host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32-in MFMA (= f32 vector) peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 / f16 MFMA: 1024 FLOP/clk/SIMD x 4 SIMD x 256 CU x 2.4 GHz (~2.5 PF)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E spec
# MFMA products per fp32 product, and the dense peak of the MFMA that executes them
ARITH = {"bf16x3": (6, BF16_MFMA_PEAK_TFLOPS, "v_mfma_f32_16x16x32_bf16"),
         "fp32": (1, FP32_MFMA_PEAK_TFLOPS, "v_mfma_f32_16x16x4_f32")}
DTYPE = {"bf16x3": "f32 via bf16x3 (x = 3 bf16 planes, 6 MFMA products, fp32 accumulate; fp32 exponent range)",
         "fp32": "f32 (exact fp32 MFMA)"}
PREC_CODE = {"fp32": 0, "bf16x3": 2}


def kernel_symbol(label, precision):
    """rocprofv3 symbol of the launch behind a profiler label (csrc/api.cpp
    ProfScope; register-staged cgemm.hip tiles are templated on the precision code)."""
    if label == "G0f_raw":
        return "tik::gcn0_kernel<1>"
    if label[:2] in ("XT", "XG", "XH") and label[2:] in ("64", "128"):
        # xgemm.hip: <BN, EPI_BIAS (0) | EPI_GRAPH (1), 4 waves per workgroup, split-K>
        return f"tik::xgemm_kernel<{label[2:]}, {1 if label[1] == 'G' else 0}, 4, {'true' if label[1] == 'H' else 'false'}>"
    if label in ("XB0", "XB1"):
        return f"tik::xblock_kernel<{'true' if label == 'XB0' else 'false'}>"
    if label[:2] == "XP" and label[2:] in ("64", "128"):
        # xgemm_pt_kernel<BN, identity, residual conv>: the label does not say which (any instantiation)
        return "tik::xgemm_pt_kernel"
    if label == "XR":
        return "tik::xgemm_splitk_reduce_kernel"
    if label == "XGW":
        return "tik::xgraph_kernel"   # <K blocks, passes>: the label does not say which (any instantiation)
    if label == "XTW":
        return "tik::xtws_kernel<1, 8, false>"
    if label == "XTWG":   # xtws + the next block's gcn (FG)
        return "tik::xtws_kernel<1, 8, true>"
    p = PREC_CODE[precision]
    nb_graph = 2 if p == 0 else 1
    cg = {"G272x64": f"272, 64, 1, 4, 1, 17, {p}, {nb_graph}", "T128x128": f"128, 128, 2, 2, 0, 0, {p}, 2",
          "T128x64": f"128, 64, 2, 2, 0, 0, {p}, 2", "T256x64": f"256, 64, 4, 1, 0, 0, {p}, 2",
          "H64x64": f"64, 64, 2, 2, 0, 0, {p}, 2"}
    return f"tik::cgemm_kernel<{cg[label]}>" if label in cg else None


def tree_profile(pattern):
    """The profiles/`pattern` summary of THIS source tree: the PMC summaries
    carry the sha256 digest of the library sources they were measured on
    (scripts/pmc_traffic.py, pmc_mfma.py; _build.source_digest), and only a
    summary whose digest equals the benchmarked tree's is used (the last by
    name when several match). Returns (path or None, reason)."""
    import glob

    from temporal_inverse_kinematics_amd._build import source_digest
    digest = source_digest()
    hits = []
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", pattern))):
        try:
            if json.load(open(p)).get("source_digest") == digest:
                hits.append(p)
        except (OSError, ValueError):
            continue
    if not hits:
        return None, f"no profiles/{pattern} was measured on this source tree (digest {digest})"
    return hits[-1], f"measured on this source tree (digest {digest})"


def _pmc_value(path, label, pattern, field, precision):
    """`field` of the kernel behind `label` in a PMC summary (scripts/pmc_traffic.py
    or pmc_mfma.py output; default: the profiles/`pattern` summary of this
    source tree, tree_profile). Returns (value or None, source path or None, note)."""
    note = "explicit path"
    if path is None:
        path, note = tree_profile(pattern)
    if not path or not os.path.exists(path):
        return None, None, note
    sym = kernel_symbol(label, precision)
    kern = json.load(open(path)).get("kernels", {})
    for k, v in kern.items():
        name = k.replace("void ", "").strip()
        if sym and (name == sym or ("<" not in sym and name.startswith(sym + "<"))):
            return v.get(field), os.path.relpath(path, REPO), note
    return None, os.path.relpath(path, REPO), note + f"; no entry for {sym}"


def _pmc_traffic(path, label, precision):
    """HBM bytes per dispatch of the kernel behind `label` (scripts/pmc_traffic.py)."""
    return _pmc_value(path, label, "*pmc_traffic*.json", "hbm_bytes_per_dispatch", precision)


def _pmc_mfma(path, label, precision):
    """MFMA-busy fraction of the kernel behind `label` (scripts/pmc_mfma.py)."""
    return _pmc_value(path, label, "*pmc_mfma*.json", "mfma_busy_frac", precision)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _one_socket_physical_cores():
    """CPUs this process may run on, restricted to the socket of the first one
    and to one hardware thread per physical core (sysfs topology)."""
    allowed = sorted(os.sched_getaffinity(0))

    def rd(c, f):
        try:
            return open(f"/sys/devices/system/cpu/cpu{c}/topology/{f}").read().strip()
        except OSError:
            return None
    pkg0 = rd(allowed[0], "physical_package_id")
    seen, cores = set(), []
    for c in allowed:
        if rd(c, "physical_package_id") != pkg0:
            continue
        key = rd(c, "core_id")
        if key in seen:
            continue
        seen.add(key)
        cores.append(c)
    return cores or allowed


def _cgroup_cpus():
    """The CPU share of this container's cgroup (cpu.max quota / period), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def _cpu_child(T: int, seconds: float):
    """The CPU baseline itself, in a child process (bench.py --cpu-child): pinned
    to the physical cores of one socket BEFORE torch is imported, so the intra-op
    threads never spread over two sockets or SMT siblings."""
    cores = _one_socket_physical_cores()
    quota = _cgroup_cpus()
    if quota is not None:   # no more cores than the cgroup's CPU share: threads past it only wait
        cores = cores[:max(1, int(quota))]
    os.sched_setaffinity(0, cores)
    import numpy as np
    import torch

    from oracle import stgcn as orc
    from temporal_inverse_kinematics_amd import synthetic as syn
    sd = syn.ik_state_dict(orc.graph_A("coco", "uniform", 2, 1), seed=0)
    nb = 64   # the reference's inference batch (inference.py:43)
    x = syn.synthetic_windows(nb, T, seed=7)
    cap = len(cores)
    cands = [n for n in (8, 16, 32, 64) if n <= cap] or [cap]
    probes = {}
    for n in cands:
        torch.set_num_threads(n)
        orc.pose_regressor_torch(x, sd)   # warm-up batch at this thread count
        t0 = time.perf_counter()
        orc.pose_regressor_torch(x, sd)
        probes[str(n)] = round(nb / (time.perf_counter() - t0), 1)
    best = int(max(probes, key=lambda k: probes[k]))
    torch.set_num_threads(best)
    rates, done_all = [], 0
    for _ in range(3):   # three windows; the median is the value
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 3:
            orc.pose_regressor_torch(x, sd)
            done += nb
        rates.append(done / (time.perf_counter() - t0))
        done_all += done
    return {"value": round(float(np.median(rates)), 1), "unit": "IK frames/s", "cores": best, "kind": "port",
            "cpu_model": _cpu_model(), "pinned_cpus": len(cores), "cgroup_cpus": quota,
            "visible_cpus": os.cpu_count(), "threads_probed": probes, "windows_rates": [round(r, 1) for r in rates],
            "sample": f"{done_all} windows (T={T}, batches of {nb}) of the reference forward restated in torch CPU ops "
                      f"(oracle/stgcn.py pose_regressor_torch, fp32 eval, pinned to the reference's fixtures), "
                      f"{best} threads pinned to {len(cores)} physical cores of one socket; median of 3 windows "
                      f"of {seconds / 3:.1f} s"}


def _cpu_baseline(T: int, seconds: float = 12.0):
    """CPU baseline (report only) in a child process, see _cpu_child."""
    import subprocess
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", "--T", str(T),
                        "--cpu-seconds", str(seconds)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"value": None, "error": r.stderr[-500:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="windows per GPU")
    ap.add_argument("--T", type=int, default=64, help="frames per window")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "fp32"],
                    help="GEMM arithmetic: bf16x3 (default; fp32 range, 6 bf16 MFMA products) or exact fp32 MFMA")
    ap.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-compare", action="store_true", help="skip the other-precision comparison runs")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the config #4 (fk) and #5 (online) measurements appended at N=1")
    ap.add_argument("--no-profile", action="store_true",
                    help="diagnostic: no per-launch HIP events in the timed region (no roofline)")
    ap.add_argument("--pmc-traffic", default=None,
                    help="PMC traffic summary (scripts/pmc_traffic.py); default: newest profiles/*pmc_traffic*.json")
    ap.add_argument("--pmc-mfma", default=None,
                    help="PMC MFMA-busy summary (scripts/pmc_mfma.py); default: newest profiles/*pmc_mfma*.json")
    args = ap.parse_args()
    if args.cpu_child:
        print(json.dumps(_cpu_child(args.T, args.cpu_seconds)))
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if rank == 0 and world > 1:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from temporal_inverse_kinematics_amd import _build, _lib, synthetic as syn
    from temporal_inverse_kinematics_amd.distributed import PosesGatherPipeline
    from temporal_inverse_kinematics_amd.inference import synthetic_model
    if rank == 0:
        _build.build()
    if world > 1:
        dist.barrier()

    B, T = args.batch, args.T
    model = synthetic_model(win_size=T, device=dev, precision=args.precision)
    reg = model.regressor
    x = torch.from_numpy(syn.synthetic_windows(B, T, seed=0, start=rank * B)).to(dev)
    Tp = reg.backbone.out_frames(T)
    full = torch.empty((world * B, Tp, 66), device=dev) if world > 1 else None

    # the all-gather of step k runs on RCCL's stream while step k+1's forward
    # runs (PosesGatherPipeline); every gather is waited on inside the timed region
    gathers = PosesGatherPipeline()

    def step():
        y = reg(x)["poses"]
        if world > 1:
            gathers.push(y, full)
        return y

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        gathers.drain()
        lib = _lib.load()
        h = reg.tik_handle()
        per_fwd = 2 * len(reg.backbone.st_gcn_networks) + 4

        def timed(k):
            """k steps between barrier + synchronize on both sides; max over ranks"""
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            gathers.drain()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            d = time.perf_counter() - t0
            if world > 1:
                tt = torch.tensor([d], device=dev, dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                d = float(tt.item())
            return d

        # timed region 1: the metric (no instrumentation: one HIP event pair per
        # launch costs ~3.5 us per event on this path, ~3.5 % of a step)
        dt = timed(args.steps)
        # timed region 2: the same K steps with a HIP event pair around every
        # launch on its stream (tik_model_profile): per-kernel durations for the roofline
        dt_prof = None
        if not args.no_profile:
            _lib.check(lib.tik_model_profile(h, per_fwd * args.steps))
            dt_prof = timed(args.steps)

        # per-kernel HIP-event timings from the timed region
        n = _lib.check(lib.tik_model_profile_count(h))
        agg, per_launch = {}, {}
        lab = ctypes.create_string_buffer(64)
        ms, fl, by = ctypes.c_float(), ctypes.c_double(), ctypes.c_double()
        for i in range(n):
            _lib.check(lib.tik_model_profile_read(h, i, lab, 64, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by)))
            full_lab = lab.value.decode()
            kern = full_lab.split(".")[0]
            a = agg.setdefault(kern, [0.0, 0, 0.0, 0.0])
            a[0] += ms.value; a[1] += 1; a[2] += fl.value; a[3] += by.value
            b = per_launch.setdefault(full_lab, [0.0, 0, 0.0, 0.0])
            b[0] += ms.value; b[1] += 1; b[2] += fl.value; b[3] += by.value
        lib.tik_model_profile(h, 0)

    # N > 1: the gathered poses of the last step are checked on rank 0 against
    # its own solve of every rank's windows (the inputs are seeded per rank)
    gather_check = None
    if world > 1:
        with torch.no_grad():
            step()
            gathers.drain()
            if rank == 0:
                xs = torch.from_numpy(np.concatenate([syn.synthetic_windows(B, T, seed=0, start=r * B)
                                                      for r in range(world)])).to(dev)
                ref = reg(xs)["poses"]
                gather_check = {"max_abs_diff_vs_rank0_solve": float((full - ref).abs().max().item()),
                                "windows": int(world * B)}
        dist.barrier()
    ms_step = dt / args.steps * 1e3
    value = world * B / (dt / args.steps)
    others = []
    if not args.no_compare:
        # the other arithmetics on the same inputs: time + max |difference| of the poses
        with torch.no_grad():
            y_main = reg(x)["poses"].clone()
            for alt in [p for p in ("fp32", "bf16x3") if p != args.precision]:
                reg.tik_precision = alt
                y_alt = reg(x)["poses"]
                for _ in range(2):
                    reg(x)
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                gathers.drain()
                torch.cuda.synchronize()
                dt_alt = time.perf_counter() - t1
                others.append({"precision": alt, "dtype": DTYPE[alt],
                               "value": round(world * B / (dt_alt / args.steps), 1),
                               "ms_per_step": round(dt_alt / args.steps * 1e3, 4),
                               "max_abs_pose_diff_vs_main": float((y_main - y_alt).abs().max().item())})
            reg.tik_precision = args.precision
    if rank == 0 and args.no_profile:
        print(json.dumps({"metric": "IK frames/sec (COCO-17->SMPLx pose)", "value": round(value, 1),
                          "ms_per_step": round(ms_step, 4), "note": "diagnostic run without per-launch events"}))
    elif rank == 0:
        dom = max(agg, key=lambda k: agg[k][0])
        tot_ms, cnt, tot_fl, tot_by = agg[dom]
        avg_s = tot_ms / cnt / 1e3
        tflops = tot_fl / cnt / avg_s / 1e12
        gbs = tot_by / cnt / avg_s / 1e9
        # the path is MFMA-bound (~36k FLOP per HBM byte). The roof
        # is the dense peak of the MFMA that executes the products: bf16x3 runs 6
        # bf16 MFMA products per fp32 product, so its fp32-equivalent peak is 2516.6/6
        # the binding roof of the dominant kernel: the larger of its fractions of
        # the MFMA roof (algorithmic FLOPs) and of the HBM roof (algorithmic bytes)
        nprod, xpeak, instr = ARITH[args.precision]
        if gbs / HBM_PEAK_GBS > tflops / (xpeak / nprod):
            bound, achieved, peak, unit = "hbm", gbs, HBM_PEAK_GBS, "GB/s"
            basis = ("HBM3E spec peak; achieved = algorithmic activation bytes (SURVEY.md §8(d)) / HIP-event "
                     "launch time (its MFMA fraction is lower)")
        else:
            bound, achieved, peak, unit = "mfma", tflops, xpeak / nprod, "TFLOP/s"
            basis = (f"{instr} dense peak {xpeak} TF / {nprod} MFMA products per fp32 product = {xpeak / nprod:.1f} "
                     f"fp32-equivalent TF; achieved = algorithmic fp32 FLOPs (SURVEY.md §8(d)) / HIP-event launch time")
        traffic, traffic_src, traffic_note = _pmc_traffic(args.pmc_traffic, dom, args.precision)
        mfma_busy, mfma_src, mfma_note = _pmc_mfma(args.pmc_mfma, dom, args.precision)
        kernels = {k: {"launches": v[1], "avg_ms": round(v[0] / v[1], 4), "share": round(v[0] / sum(a[0] for a in agg.values()), 3),
                       "tflops": round(v[2] / (v[0] / 1e3) / 1e12, 2), "gbs": round(v[3] / (v[0] / 1e3) / 1e9, 1)}
                   for k, v in agg.items()}
        fwd_flops = sum(v[2] for v in agg.values()) / args.steps
        win_bytes = T * 17 * 3 * 4 + Tp * 66 * 4
        hbm_gbs = world * B * win_bytes / (dt / args.steps) / 1e9
        out = {
            "metric": "IK frames/sec (COCO-17->SMPLx pose)",
            "value": round(value, 1),
            "unit": "IK frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "pose_rows_per_s": round(value * Tp, 1),   # windows/s x T' output rows
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPE[args.precision],
            "data": "synthetic (AMASS-shaped windows from the sample sequence; seeded synthetic weights)",
            "config": {"workload": f"ST-GCN IK forward, batch={B}x{T}-frame x COCO-17 windows per GPU -> (B,{Tp},66) "
                                   f"SMPL-X pose" + (f", RCCL all-gather of poses over {world} GPUs" if world > 1 else ""),
                       "global_batch": world * B, "window_frames": T, "out_frames": Tp,
                       "parallelism": f"dp{world}" if world > 1 else "single"},
            "roofline": {"kernel": dom, "symbol": kernel_symbol(dom, args.precision), "bound": bound,
                         "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": unit,
                         "frac": round(achieved / peak, 4), "peak_basis": basis,
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src, "traffic_note": traffic_note,
                         "mfma_busy": None if mfma_busy is None else round(mfma_busy, 4),
                         "mfma_busy_basis": "PMC SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), "
                                            "single-stream dispatches (scripts/pmc_mfma.py)",
                         "mfma_busy_source": mfma_src, "mfma_busy_note": mfma_note,
                         "algorithmic_bytes_per_launch": round(tot_by / cnt),
                         "algorithmic_flops_per_launch": round(tot_fl / cnt),
                         "avg_launch_ms": round(avg_s * 1e3, 4), "launches": cnt,
                         "executed_mfma_tflops": round(tflops * nprod, 1), "executed_mfma_peak": xpeak,
                         "activation_gbs": round(gbs, 1), "activation_hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                         "activation_basis": "the kernel's layer-to-layer activation bytes (4 B per element read "
                                             "or written once) / launch time, against the HBM3E spec peak"},
            "hbm": {"bound": "hbm", "achieved": round(hbm_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(hbm_gbs / HBM_PEAK_GBS, 6), "bytes_per_window": win_bytes,
                    "basis": "SURVEY.md §8(d) algorithmic bytes per IK frame (window in + poses out) x frames/s; "
                             "BASELINE.json's 'achieved HBM GB/s fraction' (tiny by construction: the path is "
                             "MFMA-bound)"},
            "forward": {"algorithmic_tflops": round(fwd_flops * args.steps / dt / 1e12, 2),
                        "mflop_per_window": round(fwd_flops / B / 1e6, 2), "kernels": kernels,
                        "launches": {k: {"avg_ms": round(v[0] / v[1], 4), "tflops": round(v[2] / (v[0] / 1e3) / 1e12, 1),
                                         "gbs": round(v[3] / (v[0] / 1e3) / 1e9, 0)} for k, v in per_launch.items()}},
        }
        if others:
            out["other_precisions"] = others
        if gather_check is not None:
            out["gather_check"] = gather_check
        out["profiled_ms_per_step"] = round(dt_prof / args.steps * 1e3, 4)
        out["timing"] = ("value/ms_per_step: K steps with no instrumentation; roofline/forward: a second pass of "
                         "the same K steps with HIP events around every launch on its stream")
        if world == 1 and not args.no_extras:
            # BASELINE configs #4 and #5 under the same clock (the headline stays config #2)
            from bench_fk import measure_fk
            from bench_stream import measure_online
            out["fk"] = measure_fk(batch=4096, steps=10, warmup=20)
            out["online"] = measure_online(frames=2000, warmup=100, win=T)
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = _cpu_baseline(T, args.cpu_seconds)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
