#!/bin/bash
# Full GPU test suite + smoke (what the driver runs at round end). Usage: bash scripts/gpu_tests.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-tests}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -4 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
tail -2 $OUT/smoke_$TAG.log; echo "smoke rc=$rc"; exit $rc
