#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first crash / fault / timeout (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

echo "== build"; python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; ok $rc || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1; rc=$?
tail -3 $OUT/smoke_$TAG.log; echo "smoke rc=$rc"; ok $rc || exit $rc
echo "== bench"
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
tail -c 3000 $OUT/bench_$TAG.json; echo "bench rc=$rc"; ok $rc || exit $rc
echo "== rocprofv3 kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err; rc=$?
echo "rocprof rc=$rc"; find $OUT/prof_$TAG -name "*stats*" | head
exit 0
