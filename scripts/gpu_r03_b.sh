#!/bin/bash
# round 3, step b: parity of the new bf16x3 pieces (xgemm split-K head, LDS-staged
# EPI_BIAS epilogue, two-stream split of the xgemm path), then bench A/B of each
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_b2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ik.py tests/test_gpu_precision.py tests/test_gpu_fk.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for E in TIK_X=0 TIK_XEPI=0 TIK_XEPI=2 TIK_SPLIT=0 TIK_XHEAD_KS=0 TIK_XHEAD_KS=8 TIK_SPLIT_LAG=1 TIK_SPLIT_LAG=3 TIK_XSTAGGER=2 TIK_XSTAGGER=4 TIK_SPLIT=0,TIK_XSTAGGER=4; do
  env ${E//,/ } timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-compare --no-cpu-baseline > $OUT/bench_${TAG}_$E$r.json 2> $OUT/bench_${TAG}_$E$r.err || exit 4
  python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_$E$r.json')); L=d['forward']['launches']
print('$r $E value', d['value'], 'ms', d['ms_per_step'], 'prof_ms', d['profiled_ms_per_step'], 'sum_launch_ms', round(sum(v['avg_ms'] for v in L.values()),4))
if '$r' == '1': print('   ', ' '.join(f\"{k}={v['avg_ms']}\" for k,v in sorted(L.items())))
"
done; done
for E in TIK_X=0 TIK_FK_XGEMM=0; do
  env $E timeout -k 10 300 python bench_fk.py --cpu-seconds 1 > $OUT/fk_${TAG}_$E.json 2> $OUT/fk_${TAG}_$E.err || exit 5
  echo "fk $E $(cut -c1-400 $OUT/fk_${TAG}_$E.json)"
done
