#!/bin/bash
# Component-cost experiment on the temporal convs: the diagnostic build
# (scripts/bin/libtik_tune.so, -DTIK_XTUNE) with parts switched off per TIK_XTUNE
# bits (WS kernel: 1 A DMA, 2 B DMA, 4 MFMAs, 8 split, 16 stores; XT kernel: 1 A, 2 B, 8 split).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TIK_LIB=scripts/bin/libtik_tune.so
OUT=gpurun_out; TAG=${1:-tune}; shift
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --no-compare --no-cpu-baseline --no-extras --steps 10 --warmup 3 > $OUT/${TAG}.json 2> $OUT/${TAG}.err || { echo "[$cfg] failed"; tail -3 $OUT/${TAG}.err; exit 3; }
  python - "$OUT/${TAG}.json" "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["forward"]["launches"]
sel = {k: v["avg_ms"] for k, v in L.items() if k.split(".")[1] in ("L3", "L6") and k[:2] in ("XW", "XT", "XG")}
print(f"[{sys.argv[2]:28s}] step {d['ms_per_step']:.3f} ms  " + "  ".join(f"{k} {v:.4f}" for k, v in sel.items()))
PY
done
