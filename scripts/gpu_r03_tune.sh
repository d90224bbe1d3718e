#!/bin/bash
# component-cost experiments: bench + trace of the ping-pong xgemm with parts switched off (TIK_XTUNE bits)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp TIK_XPP=1
OUT=gpurun_out; TAG=${1:-r03_tune}; mkdir -p $OUT
for t in 0 3 4 8 12 16 15 31; do
  TIK_XTUNE=$t TIK_X_TRACE=1 timeout -k 10 120 python scripts/xtrace.py > /dev/null 2> $OUT/xtrace_${TAG}_$t.txt || exit 3
  echo "== tune $t"; sed -n '/traced forward/,$p' $OUT/xtrace_${TAG}_$t.txt | grep "XT128.L3\|XG128.L3"
done
