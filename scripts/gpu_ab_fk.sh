#!/bin/bash
# FK tests + A/B of the FK step under environment settings (one bench_fk per setting).
# Usage: bash scripts/gpu_ab_fk.sh TAG "ENV=a" "ENV=b" ...   ("-" = no extra env)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift; mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build_$TAG.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_fk.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 300 python bench_fk.py --cpu-seconds 0.5 > $OUT/abfk_${TAG}_$i.json 2> $OUT/abfk_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/abfk_${TAG}_$i.json'));k=d['kernels'];print('$cfg', d['value'], d['ms_per_step'], {n:round(v['avg_ms'],4) for n,v in k.items()})"
done
