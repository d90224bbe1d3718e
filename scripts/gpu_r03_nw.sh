#!/bin/bash
# A/B of the xgemm wave count on one box: TIK_XNW=4 parity subset + bench + trace, then TIK_XNW=8 bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_nw}; mkdir -p $OUT
TIK_XNW=4 bash scripts/gpu_r03_qt.sh ${TAG}_nw4 || exit $?
TIK_XNW=8 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-compare --no-cpu-baseline > $OUT/bench_${TAG}_nw8.json 2> $OUT/bench_${TAG}_nw8.err || exit 4
python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_nw8.json'))
print('nw8 value', d['value'], 'ms', d['ms_per_step'])
for k,v in d['forward']['launches'].items(): print(' ', k, v)
"
