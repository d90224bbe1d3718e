#!/bin/bash
# FK blend GEMM tile order A/B (TIK_FK_GM: 1 = rows outer, the round-4 order; auto = one row group per XCD)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fk.py > gpurun_out/fk_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/fk_pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in "TIK_FK_GM=1" "-" "TIK_FK_GM=2" "TIK_FK_GM=8" "TIK_FK_GM=1" "-"; do
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 200 python bench_fk.py --cpu-seconds 0 > gpurun_out/fk_ab.json 2> gpurun_out/fk_ab.err || { tail -5 gpurun_out/fk_ab.err; exit 3; }
  python - gpurun_out/fk_ab.json "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]:24s}] {d['value']:.0f} bodies/s  {d['ms_per_step']:.4f} ms  " + "  ".join(f"{k} {v['avg_ms']:.4f}" for k, v in d["kernels"].items()))
PY
done
