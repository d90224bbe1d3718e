#!/bin/bash
# r06 fktrace: kernel timeline of the FK step (two streams) from rocprofv3 --kernel-trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/fktrace -o fk -- python3 bench_fk.py --steps 3 --warmup 5 --cpu-seconds 0.1 > $O/fktrace.log 2>&1 || { tail -20 $O/fktrace.log; exit 1; }
f=$(find $O/fktrace -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY' | tee $O/fktrace_timeline.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the 3 timed FK steps (5 warmup steps before them, 3 profiled ones after)
ch = [i for i, r in enumerate(rows) if "fk_chain" in r["Kernel_Name"]]
i0, i1 = ch[-6], ch[-3]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%9.1f %9.1f %8.1f q%s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r.get("Queue_Id", "?"), r["Kernel_Name"][:70]))
PY
