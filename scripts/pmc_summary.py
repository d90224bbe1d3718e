"""Summarise rocprofv3 --pmc passes (counter_collection.csv) per (kernel, grid):
average counter value per dispatch.  usage: pmc_summary.py <dir-glob> [name-filter]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void tik::", "").replace("tik::", "")
    return name[:60]


def main():
    dirs = sorted(glob.glob(sys.argv[1]))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), int(r.get("Grid_Size", 0) or 0))
                if filt and filt not in k[0]:
                    continue
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        vals = " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(acc[k].items()))
        print(f"{k[0]:<60} grid={k[1]:<9} {vals}")


if __name__ == "__main__":
    main()
