#!/bin/bash
# robust A/B on one box: parity subset with env A, then benches A B A B (30 steps each);
# prints wall value and the sum of per-launch HIP-event times per run
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; A=${2:-X=0}; B=${3:-X=0}; mkdir -p $OUT
env $A timeout -k 10 400 python -u -m pytest tests/test_gpu_ik.py tests/test_gpu_precision.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16x3 or precision or moveai" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -2 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in A B; do
  [ $v = A ] && E=$A || E=$B
  env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-compare --no-cpu-baseline > $OUT/bench_${TAG}_$v$r.json 2> $OUT/bench_${TAG}_$v$r.err || exit 4
  python -c "
import json; d=json.load(open('$OUT/bench_${TAG}_$v$r.json')); L=d['forward']['launches']
top=sorted(L.items(), key=lambda kv: kv[0])
print('$v$r ($E) value', d['value'], 'ms', d['ms_per_step'], 'sum_launch_ms', round(sum(v['avg_ms'] for v in L.values()),4))
if '$r' == '1': print('   ', ' '.join(f\"{k}={v['avg_ms']}\" for k,v in top))
"
done; done
