#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "xblock or model_vs_golden or batch_invariant" > gpurun_out/xb2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/xb2_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xb2 "-" "TIK_XBLK=0" && bash scripts/gpu_r04_xgtrace.sh | grep XB
