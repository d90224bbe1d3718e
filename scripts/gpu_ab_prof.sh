#!/bin/bash
# A/B of the IK step under environment settings with the per-kernel HIP-event
# profile (forward.kernels). Usage: bash scripts/gpu_ab_prof.sh TAG "ENV=a" "-" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift; mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras --steps 30 > $OUT/abp_${TAG}_$i.json 2> $OUT/abp_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/abp_${TAG}_$i.json'));k=d.get('forward',{}).get('kernels') or d.get('kernels',{});print('$cfg', d['value'], d['ms_per_step'], {n:round(v['avg_ms'],4) for n,v in k.items()})"
done
