#!/bin/bash
# Same-box A/B over several builds of libtik.so: "new" = the in-tree library,
# any other name = ab/libtik_<name>.so (scripts/build_base.sh, or a copy built
# with TIK_HIPCC_FLAGS). Parity of each non-base build first (AB_TESTS=1), then
# $ROUNDS rounds of the bench alternating the builds.
#   gpu_ab_libs.sh TAG base new xorder ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/ab_$TAG; mkdir -p $O
# a spec is NAME or NAME:VAR=VALUE[,VAR=VALUE] (the build, plus environment for its runs)
lib() { local n=${1%%:*}; [ "$n" = new ] && echo "" || echo "ab/libtik_$n.so"; }
envs() { [[ "$1" == *:* ]] && echo "${1#*:}" | tr ',' ' ' || echo "TIK_AB=1"; }
if [ -n "${AB_TESTS:-}" ]; then
  for v in "$@"; do
    [ "$v" = base ] && continue
    env $(envs $v) TIK_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_ik.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${AB_K:-bf16x3}" > $O/pt_$v.log 2>&1; rc=$?
    echo "pytest $v: $(tail -1 $O/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    env $(envs $v) TIK_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v$r.json'));l=d['forward']['launches'];print('$v$r', d['value'], d['ms_per_step'], 'prof', d['profiled_ms_per_step'], ' '.join(f'{k}={v[\"avg_ms\"]}' for k,v in sorted(l.items()) if k.startswith('XG')))"
  done
done
