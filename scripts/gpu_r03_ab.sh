#!/bin/bash
# A/B on one box: parity subset + bench + trace with env "$2" (e.g. TIK_XPP=1), then bench with env "$3"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_ab}; A=${2:-TIK_XPP=1}; B=${3:-TIK_XPP=0}; mkdir -p $OUT
env $A bash scripts/gpu_r03_qt.sh ${TAG}_a || exit $?
env $B timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-compare --no-cpu-baseline > $OUT/bench_${TAG}_b.json 2> $OUT/bench_${TAG}_b.err || exit 4
python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_b.json'))
print('B value', d['value'], 'ms', d['ms_per_step'])
for k,v in d['forward']['launches'].items(): print(' ', k, v)
"
