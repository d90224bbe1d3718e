#!/bin/bash
# quick loop: bf16x3 parity subset + bench (no comparisons, short CPU baseline)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_q}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ik.py tests/test_gpu_precision.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16x3 or precision or moveai" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-compare --no-cpu-baseline > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
python -c "
import json; d=json.load(open('$OUT/bench_$TAG.json'))
print('value', d['value'], 'ms', d['ms_per_step'])
for k,v in d['forward']['launches'].items(): print(' ', k, v)
"; echo "bench rc=$rc"
