#!/bin/bash
# Online IK latency under environment settings (bench_stream per setting).
# Usage: bash scripts/gpu_online_ab.sh TAG "ENV=a" "ENV=b" ...   ("-" = no extra env)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift; mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build_$TAG.log 2>&1 || exit 2
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 200 python bench_stream.py --frames 3000 > $OUT/abon_${TAG}_$i.json 2> $OUT/abon_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/abon_${TAG}_$i.json'));print('$cfg', d['value'], d['p99_us'])"
done
