#!/bin/bash
# xtws: no barrier at a tile's first K block (default) vs the barrier kept (build scripts/bin/libtik_xweb.so with -DXW_EPIBAR=0)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TIK_LIB=scripts/bin/libtik_xweb.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ik.py -k "xtws or golden or ragged" > gpurun_out/xweb_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/xweb_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xweb "-" "TIK_LIB=scripts/bin/libtik_xweb.so" "-" "TIK_LIB=scripts/bin/libtik_xweb.so"
