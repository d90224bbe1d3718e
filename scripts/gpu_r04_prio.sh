#!/bin/bash
# Static s_setprio for waves 4-7 of the 8-wave persistent kernels (scripts/bin/libtik_prio.so, -DTIK_YPRIO=1) vs default
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TIK_LIB=scripts/bin/libtik_prio.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ik.py -k "xgraph or xblock or xtws" > gpurun_out/prio_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/prio_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh prio "-" "TIK_LIB=scripts/bin/libtik_prio.so" "-" "TIK_LIB=scripts/bin/libtik_prio.so" "TIK_XTWS=24" "TIK_XTWS=24 TIK_LIB=scripts/bin/libtik_prio.so"
