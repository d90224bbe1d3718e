"""Mean of every counter per kernel over one rocprofv3 --pmc pass (kernel trace
only), with SQ wait/active shares of SQ_WAVE_CYCLES when those were collected.

    python scripts/pmc_generic.py <pass-dir> [kernel-substring]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            if sub in name:
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(vals.items()):
        m = {n: sum(v) / len(v) for n, v in c.items()}
        n = max(len(v) for v in c.values())
        line = " ".join(f"{n_}={v:.4g}" for n_, v in sorted(m.items()))
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            line += " | " + " ".join(f"{n_[3:]}/WAVE={m[n_] / wc:.3f}" for n_ in
                                     ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS") if n_ in m)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            line += f" | mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
        print(f"{k[:64]:<64} n={n} {line}")


if __name__ == "__main__":
    main()
