#!/bin/bash
# xtws as the L3/L4 default: the whole GPU suite, then a same-box A/B against XT128 (TIK_XTWS=0)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/xtwdef_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/xtwdef_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xtwdef "-" "TIK_XTWS=0" "-" "TIK_XTWS=0"
