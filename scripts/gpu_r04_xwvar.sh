#!/bin/bash
# xtws variants: D=2 register prefetch (scripts/bin/libtik_xwd2.so), split units early in the block (libtik_xwsa.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in xwd2 xwsa; do
  TIK_LIB=scripts/bin/libtik_$L.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ik.py -k xtws > gpurun_out/xwvar_$L.log 2>&1; rc=$?
  tail -1 gpurun_out/xwvar_$L.log; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r04_ab.sh xwvar "-" "TIK_LIB=scripts/bin/libtik_xwd2.so" "TIK_LIB=scripts/bin/libtik_xwsa.so" "-" "TIK_LIB=scripts/bin/libtik_xwd2.so" "TIK_LIB=scripts/bin/libtik_xwsa.so"
