#!/bin/bash
# xgraph.hip phase trace (diagnostic build scripts/bin/libtik_trace.so, -DTIK_XTRACE)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TIK_LIB=scripts/bin/libtik_trace.so TIK_X_TRACE=1 timeout -k 10 300 python bench.py --no-compare --no-cpu-baseline --no-extras --steps 2 --warmup 1 > gpurun_out/xgtrace.json 2> gpurun_out/xgtrace.err; rc=$?
grep -E "XGTRACE|XBTRACE" gpurun_out/xgtrace.err | tail -24
exit $rc
