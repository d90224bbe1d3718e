#!/bin/bash
# Training-step session: GPU parity tests of the trainer, the training bench,
# and a rocprofv3 kernel-stats pass of the bench. Usage: bash scripts/gpu_train.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${1:-train}
mkdir -p $OUT
echo "== pytest train"

timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_train_$TAG.log 2>&1; rc=$?
tail -15 $OUT/pytest_train_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== bench_train"
timeout -k 10 300 python bench_train.py > $OUT/bench_train_$TAG.json 2> $OUT/bench_train_$TAG.err; rc=$?
cat $OUT/bench_train_$TAG.json; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_train_$TAG -o run -- python bench_train.py --steps 20 --no-cpu-baseline > /dev/null 2> $OUT/prof_train_$TAG.err; rc=$?
echo "prof rc=$rc"
head -25 $OUT/prof_train_$TAG/run_kernel_stats.csv | cut -c1-160
exit $rc
