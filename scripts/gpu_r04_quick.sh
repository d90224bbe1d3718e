#!/bin/bash
# Quick GPU iteration: a selected parity subset (-k expression), then a short bench line.
#   bash scripts/gpu_r04_quick.sh TAG "pytest -k expression" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-q}; KEXPR=${2:-xgraph}
shift 2 || true
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 300 python bench.py --no-compare --no-cpu-baseline --no-extras "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
python - "$OUT/bench_$TAG.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "prof_ms", d.get("profiled_ms_per_step"), "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["forward"]["launches"].items(): print(f"  {k:16s} {v['avg_ms']:.4f} ms {v['tflops']:7.1f} TF {v['gbs']:7.0f} GB/s")
PY
echo "bench rc=$rc"; exit $rc
