#!/bin/bash
# xgemm two-stream split A/B: split parity tests, then the bench with the
# split off, on (parts together) and with part 1 lagging part 0 by L launches
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-split}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ik.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_stream" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -2 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for E in TIK_SPLIT=0 TIK_SPLIT_LAG=0 TIK_SPLIT_LAG=1 TIK_SPLIT_LAG=2 TIK_SPLIT_LAG=3 TIK_SPLIT_LAG=4 TIK_SPLIT_N=3; do
  env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-compare --no-cpu-baseline --no-profile > $OUT/bench_${TAG}_$E$r.json 2> $OUT/bench_${TAG}_$E$r.err || exit 4
  echo "$r $E $(cat $OUT/bench_${TAG}_$E$r.json)"
done; done
