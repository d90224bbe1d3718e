#!/bin/bash
# Quick GPU iteration: selected GPU tests (pytest -k expression, default all GPU
# tests of the given files) + optional benches. Usage:
#   bash scripts/gpu_quick.sh TAG "tests/test_gpu_fk.py" [bench|fk|ik|all]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; FILES=$2; WHAT=${3:-none}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build_$TAG.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -5 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
if [ "$WHAT" = fk ] || [ "$WHAT" = all ]; then
  timeout -k 10 300 python bench_fk.py --cpu-seconds 1 > $OUT/fk_$TAG.json 2> $OUT/fk_$TAG.err; rc=$?
  cat $OUT/fk_$TAG.json; echo "fk rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "$WHAT" = ik ] || [ "$WHAT" = all ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
  python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'],d['ms_per_step']);[print(k,v) for k,v in d['forward']['launches'].items()]"; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
