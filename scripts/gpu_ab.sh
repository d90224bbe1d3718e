#!/bin/bash
# A/B of the IK forward step under environment settings (one bench per setting).
# Usage: bash scripts/gpu_ab.sh TAG "ENV=a ENV2=b" "ENV=c" ...   ("-" = no extra env)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift; mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build_$TAG.log 2>&1 || exit 2
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras --no-profile --steps 30 > $OUT/ab_${TAG}_$i.json 2> $OUT/ab_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/ab_${TAG}_$i.json'));print('$cfg', d['value'], d['ms_per_step'])"
done
