#!/bin/bash
# Round 6: fused xtws + next-block gcn parity tests, then a same-box A/B of the
# IK step: fused (in-tree libtik.so), fused with one gcn weight register set
# (scripts/bin/libtik_swg.so), separate XTW + XGW launches (TIK_XFG=0).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-ab3}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ik.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "xtws_fused or xtws_vs_tiled or xgraph_vs_tiled or model_vs_golden or batch_invariant" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for cfg in "TIK_XFG=0" "-" "TIK_LIB=scripts/bin/libtik_swg.so" "TIK_XFG=0" "-" "TIK_LIB=scripts/bin/libtik_swg.so"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras --steps 30 > $OUT/ab_${TAG}_$i.json 2> $OUT/ab_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/ab_${TAG}_$i.json'));k=d.get('forward',{}).get('launches',{});print('$cfg', d['value'], d['ms_per_step'], {n:v['avg_ms'] for n,v in k.items() if n[:2] in ('XT','XG')})"
done
