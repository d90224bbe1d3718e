#!/bin/bash
# Same-box A/B of env settings on the bench line (short runs, no compare / cpu / extras).
#   bash scripts/gpu_r04_ab.sh TAG "ENV1" "ENV2" ...   (each ENV a space-separated VAR=VALUE list, "-" = none)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=$1; shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --no-compare --no-cpu-baseline --no-extras --steps 20 > $OUT/ab_${TAG}_$i.json 2> $OUT/ab_${TAG}_$i.err; rc=$?
  [ $rc -eq 0 ] || { echo "config $i ($cfg) rc=$rc"; tail -5 $OUT/ab_${TAG}_$i.err; exit $rc; }
  python - "$OUT/ab_${TAG}_$i.json" "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(f"[{sys.argv[2]}] value {d['value']} ms {d['ms_per_step']} prof_ms {d.get('profiled_ms_per_step')} roof {d['roofline']['kernel']} {d['roofline']['frac']}")
for k, v in d["forward"]["launches"].items(): print(f"  {k:16s} {v['avg_ms']:.4f} ms {v['tflops']:7.1f} TF {v['gbs']:7.0f} GB/s")
PY
done
