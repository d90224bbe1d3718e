#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xgemm_ws or model_vs_golden" > gpurun_out/pytest_ws1.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ws1.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh ws1 "-" "TIK_XWS_S=3" "TIK_XWS=0"
