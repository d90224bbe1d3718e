#!/bin/bash
# rocprofv3 kernel trace of the FK bench (per-kernel durations and the gaps between them)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fkprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fkprof -o fk -- python3 bench_fk.py --cpu-seconds 0 --steps 10 > gpurun_out/fkprof/bench.json 2> gpurun_out/fkprof/bench.err || { tail -5 gpurun_out/fkprof/bench.err; exit 3; }
f=$(find gpurun_out/fkprof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 40 kernels: print name, duration, gap to the previous end
prev = None
for r in rows[-44:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{r['Kernel_Name'][:60]:60s} dur {(e - s) / 1e3:8.1f} us  gap {gap:7.1f} us")
    prev = e
PY
