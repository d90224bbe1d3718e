"""MFMA busy fraction per kernel dispatch from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (kernel-trace only).

GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS note), so
a dispatch lasts GRBM_GUI_ACTIVE / 8 shader cycles; SQ_VALU_MFMA_BUSY_CYCLES
counts SIMD cycles with an MFMA in flight (32 per 32x32x16 MFMA, 16 per
16x16x32), summed over the chip. busy_frac = busy / (cycles x SIMDs).

    python scripts/pmc_mfma.py <pass-dir> <out.json> [n_simd=1024]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from temporal_inverse_kinematics_amd._build import source_digest  # noqa: E402


def main():
    d, out = sys.argv[1:3]
    nsimd = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, c in sorted(vals.items()):
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", []), c.get("GRBM_GUI_ACTIVE", [])
        if not busy or not gui:
            continue
        b, g = sum(busy) / len(busy), sum(gui) / len(gui)
        cyc = g / 8.0
        res[k] = {"dispatches": len(busy), "mfma_busy_cycles_per_dispatch": b, "gui_active_per_dispatch": g,
                  "kernel_cycles": cyc, "mfma_busy_frac": b / (cyc * nsimd) if cyc > 0 else None}
    json.dump({"source_digest": source_digest(), "method": "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE on "
                         "'bench.py --steps 3 --warmup 1'; busy / (GRBM_GUI_ACTIVE / 8 x %d SIMDs)" % nsimd,
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k[:70]:<70} n={v['dispatches']:4d} busy={v['mfma_busy_cycles_per_dispatch']:.3e} "
              f"cyc={v['kernel_cycles']:.3e} frac={v['mfma_busy_frac']:.3f}")


if __name__ == "__main__":
    main()
