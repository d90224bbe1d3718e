#!/bin/bash
# quick loop + trace: bf16x3 parity subset, bench, one traced forward
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_qt}; mkdir -p $OUT
bash scripts/gpu_r03_q.sh $TAG || exit $?
TIK_X_TRACE=1 timeout -k 10 120 python scripts/xtrace.py > /dev/null 2> $OUT/xtrace_$TAG.txt || exit 3
sed -n '/traced forward/,$p' $OUT/xtrace_$TAG.txt | grep XTRACE
