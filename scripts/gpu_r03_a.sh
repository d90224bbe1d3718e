#!/bin/bash
# round 3, bf16x3 pass: precision tests, IK parity for bf16x3, boundary tests, quick bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_ik.py tests/test_gpu_stream.py tests/test_gpu_fk.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "precision or bf16x3 or stggcn18 or checkpoint or timeout or concurrent or fk or smplx" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -5 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
head -c 3000 $OUT/bench_$TAG.json; echo "bench rc=$rc"
