#!/bin/bash
# xtconv.hip check: bitwise vs the tiled temporal conv, then same-box A/B on the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "xtconv" > gpurun_out/xtc_pytest.log 2>&1; rc=$?
tail -10 gpurun_out/xtc_pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab.sh xtc "TIK_XTC=255" "TIK_XTC=0"
