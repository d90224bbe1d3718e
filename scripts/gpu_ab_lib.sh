#!/bin/bash
# A/B of two builds of libtik.so on one box: the in-tree library (new) against
# another build (old, e.g. scripts/bin/libtik_old.so built from the previous
# commit). Runs the IK GPU tests on the new build, then alternating benches
# with the per-kernel HIP-event profile, then a FETCH_SIZE pass of each
# (single-stream, kernel-trace only).
# Usage: bash scripts/gpu_ab_lib.sh TAG OLD_LIB [pytest file]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; OLD=$2; TESTS=${3:-tests/test_gpu_ik.py}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for lib in "$OLD" "" "$OLD" ""; do
  i=$((i + 1))
  name=${lib:-new}
  TIK_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras --steps 30 > $OUT/ablib_${TAG}_$i.json 2> $OUT/ablib_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/ablib_${TAG}_$i.json'));k=d.get('forward',{}).get('kernels') or d.get('kernels',{});print('$name', d['value'], d['ms_per_step'], {n:round(v['avg_ms'],4) for n,v in k.items()})"
done
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare --no-extras"
for lib in "$OLD" ""; do
  name=$([ -n "$lib" ] && echo old || echo new)
  TIK_SPLIT=0 TIK_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/abfetch_${TAG}_$name -o run -- $B > /dev/null 2> $OUT/abfetch_${TAG}_$name.err || exit $?
done
python scripts/pmc_generic.py $OUT/abfetch_${TAG}_old > $OUT/abfetch_${TAG}.txt 2>&1
python scripts/pmc_generic.py $OUT/abfetch_${TAG}_new >> $OUT/abfetch_${TAG}.txt 2>&1
cat $OUT/abfetch_${TAG}.txt
