#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 300 --timeout-method thread -k "xblock or model_vs_golden or ragged or batch_invariant" > gpurun_out/pytest_xb.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_xb.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xb "-" "TIK_XBLK=0"
