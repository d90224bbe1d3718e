#!/bin/bash
# xtws.hip (weight-stationary halo temporal conv, TIK_XTWS) : tests, then a same-box A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ik.py -k "xtws" > gpurun_out/xtws_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/xtws_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xtws "-" "TIK_XTWS=24" "-" "TIK_XTWS=24"
