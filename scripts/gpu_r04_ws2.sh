#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xgemm_ws" > gpurun_out/pytest_ws2.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ws2.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh ws2 "-" "TIK_XWS=0" || exit 3
export TIK_LIB=scripts/bin/libtik_trace.so TIK_X_TRACE=1 TIK_SPLIT=0
timeout -k 10 200 python scripts/xtrace.py > gpurun_out/wstrace2.out 2> gpurun_out/wstrace2.txt
grep -A30 "traced forward" gpurun_out/wstrace2.txt | grep "TRACE.*L[36]"
