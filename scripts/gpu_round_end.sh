#!/bin/bash
# Round-end GPU session: parity tests, smoke, full bench, rocprofv3 kernel
# stats of the bench, and the two PMC traffic passes (FETCH_SIZE, WRITE_SIZE,
# separately, kernel-trace only). Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ]; }
PHASE=${2:-all}   # tests | measure | all
echo "== build"; python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
if [ "$PHASE" != measure ]; then
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; ok $rc || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
tail -2 $OUT/smoke_$TAG.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
[ "$PHASE" = tests ] && exit 0
echo "== pmc passes + kernel stats (single-stream)"
bash scripts/gpu_pmc_all.sh $TAG; rc=$?
echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 400 python bench.py --pmc-traffic $OUT/pmc_traffic_$TAG.json --pmc-mfma $OUT/pmc_mfma_$TAG.json > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
tail -c 1500 $OUT/bench_$TAG.json; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== stream"
timeout -k 10 300 python bench_stream.py --frames 3000 > $OUT/stream_$TAG.json 2> $OUT/stream_$TAG.err; rc=$?
cat $OUT/stream_$TAG.json; echo "stream rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== fk"
timeout -k 10 300 python bench_fk.py > $OUT/fk_$TAG.json 2> $OUT/fk_$TAG.err; rc=$?
cat $OUT/fk_$TAG.json; echo "fk rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== train"
timeout -k 10 300 python bench_train.py > $OUT/train_$TAG.json 2> $OUT/train_$TAG.err; rc=$?
cat $OUT/train_$TAG.json; echo "train rc=$rc"
exit 0
