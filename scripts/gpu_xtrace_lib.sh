#!/bin/bash
# Per-phase xgemm timing (prologue / K loop / identity / epilogue cycles per
# workgroup) from a -DTIK_XTRACE build of the library: ab/libtik_xtrace.so
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; TAG=${1:-xt}
TIK_LIB=ab/libtik_xtrace.so TIK_X_TRACE=1 TIK_SPLIT=0 timeout -k 10 120 python scripts/xtrace.py > $O/xtrace_$TAG.out 2> $O/xtrace_$TAG.txt || exit $?
grep XTRACE $O/xtrace_$TAG.txt | tail -19
