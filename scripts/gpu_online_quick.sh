#!/bin/bash
# online IK: stream tests + bench_stream + per-phase trace. Usage: bash scripts/gpu_online_quick.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; TAG=$1; mkdir -p $O
python -m temporal_inverse_kinematics_amd._build > $O/build_$TAG.log 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1; rc=$?
tail -3 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench_stream.py --frames 3000 > $O/stream_$TAG.json 2> $O/stream_$TAG.err || exit $?
cat $O/stream_$TAG.json
timeout -k 10 200 python scripts/online_trace.py > $O/online_trace_$TAG.txt 2>&1 || exit $?
cat $O/online_trace_$TAG.txt
