#!/bin/bash
# A/B of the trainer's reduction knobs on one box: bench_train under env settings
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for cfg in "" "TIK_CS_ROWS=256" "TIK_CS_ROWS=64" "TIK_WG_TARGET=256" "TIK_WG_TARGET=1024" ""; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python bench_train.py --no-cpu-baseline --steps 100 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
done
