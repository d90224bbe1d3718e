#!/bin/bash
# xgraph.hip check: bitwise vs tiled G, then same-box A/B on the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "xgraph or xblock_whole" > gpurun_out/xgw_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/xgw_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xgw "-" "TIK_XGW=0"
