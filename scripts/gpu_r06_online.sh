#!/bin/bash
# Round 6: online IK with layer 0's gcn inside its temporal-conv tasks — the
# stream tests, then p50 alternating against the G0-phase step (TIK_ONLINE_L0G=0).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-onl}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for cfg in "TIK_ONLINE_L0G=0" "-" "TIK_ONLINE_L0G=0" "-"; do
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 200 python bench_stream.py --frames 3000 > $OUT/abonl_${TAG}.json 2>> $OUT/abonl_${TAG}.err || exit $?
  python -c "import json;d=json.load(open('$OUT/abonl_${TAG}.json'));print('$cfg', d.get('value'), d.get('p99_us'))"
done
