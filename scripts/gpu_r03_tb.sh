#!/bin/bash
# wall-clock bench per (TIK_XPP, TIK_XTUNE) pair: "pp:tune" arguments
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift; mkdir -p $OUT
for c in "$@"; do
  pp=${c%%:*}; t=${c##*:}
  TIK_XPP=$pp TIK_XTUNE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-compare --no-cpu-baseline > $OUT/bench_${TAG}_${pp}_${t}.json 2> $OUT/bench_${TAG}_${pp}_${t}.err || exit 4
  python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_${pp}_${t}.json'))
L=d['forward']['launches']
print('pp $pp tune $t value', d['value'], 'ms', d['ms_per_step'], 'XT128.L3', L['XT128.L3']['avg_ms'], 'XG128.L3', L['XG128.L3']['avg_ms'])
"
done
