#!/bin/bash
# FK: GPU parity tests, then the FK bench line with the sparse skinning kernel and with the dense GEMM
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fk.py > gpurun_out/fk_pytest.log 2>&1; rc=$?
tail -6 gpurun_out/fk_pytest.log
[ $rc -eq 0 ] || exit $rc
for sp in 1 0; do
  TIK_FK_SPARSE=$sp timeout -k 10 200 python bench_fk.py --cpu-seconds 0 > gpurun_out/fk_sp$sp.json 2> gpurun_out/fk_sp$sp.err || { tail -5 gpurun_out/fk_sp$sp.err; exit 3; }
  python - gpurun_out/fk_sp$sp.json $sp <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[sparse={sys.argv[2]}] {d['value']:.0f} bodies/s  {d['ms_per_step']:.4f} ms  " + "  ".join(f"{k} {v['avg_ms']:.4f}" for k, v in d["kernels"].items()))
PY
done
