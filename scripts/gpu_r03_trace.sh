#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_trace}; mkdir -p $OUT
for t in 0 3; do
  TIK_X_TRACE=1 TIK_XTUNE=$t timeout -k 10 120 python scripts/xtrace.py > /dev/null 2> $OUT/xtrace_${TAG}_$t.txt || exit 3
  echo "tune $t"; sed -n '/traced forward/,$p' $OUT/xtrace_${TAG}_$t.txt | grep XTRACE
done
