#!/bin/bash
# Round-4 check: GPU parity tests, then the bench line (with the fk/online keys).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r04}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --cpu-seconds 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
tail -c 600 $OUT/bench_$TAG.json; echo "bench rc=$rc"; exit $rc
