#!/bin/bash
# Root-cause bisection of the round-1 concurrency-only corruption:
# builds of the pre-fix tree 283cbfa with subsets of the fix (bisect/, made and
# described by scripts/make_bisect.sh). Each: 4 handles on 4 streams x 12 reps
# vs serial, then 4 processes x 300 reps. Usage: gpu_bisect.sh [variants...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/bisect; mkdir -p $O
for v in ${@:-v0 v1 v2}; do
  (cd bisect/$v && timeout -k 10 120 python scripts/diag_streams.py 4 12 > $O/s4_$v.json 2> $O/s4_$v.err) || exit 3
  echo "$v streams: $(python -c "import json;d=json.load(open('$O/s4_$v.json'));print(max(d['max_diff_per_rep']), sum(x>0 for x in d['max_diff_per_rep']), 'of', len(d['max_diff_per_rep']))")"
  (cd bisect/$v && timeout -k 10 240 python scripts/diag_mproc.py 4 > $O/mp_$v.json 2> $O/mp_$v.err) || exit 4
  echo "$v procs: $(cat $O/mp_$v.json)"
done
