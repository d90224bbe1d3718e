#!/bin/bash
# sub-batch sweep (TIK_DMA_CHUNK = windows per xgemm sub-batch): MALL residency of the layer tensors
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_chunk}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bf16x3" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -2 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for c in 0 512 256 128; do
  TIK_DMA_CHUNK=$c timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-compare --no-cpu-baseline > $OUT/chunk_${TAG}_$c.json 2>/dev/null || exit 3
  python -c "
import json; d=json.load(open('$OUT/chunk_${TAG}_$c.json'))
print('chunk $c', d['value'], d['ms_per_step'], 'prof', d['profiled_ms_per_step'], ' '.join(f\"{k}={v['avg_ms']:.3f}\" for k,v in d['forward']['launches'].items() if k.startswith('X')))
"
done
