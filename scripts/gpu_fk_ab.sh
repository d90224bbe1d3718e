#!/bin/bash
# FK (config #4): parity tests, then bench_fk with both GEMMs on xgemm (default)
# vs the register-staged GEMMs (TIK_FK_XGEMM=0), and a rocprofv3 kernel-stats pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; TAG=${1:-fk}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fk.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_fk_$TAG.log 2>&1; rc=$?
tail -2 $O/pytest_fk_$TAG.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for E in TIK_AB=1 TIK_FK_PT=0 TIK_FK_XGEMM=0; do
  env $E timeout -k 10 200 python bench_fk.py --cpu-seconds 1 > $O/fk_${TAG}_$E$r.json 2> $O/fk_${TAG}_$E$r.err || exit 4
  python -c "import json;d=json.load(open('$O/fk_${TAG}_$E$r.json'));print('$E$r', d['value'], d['ms_per_step'], d['gemm_tflops'])"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fk_$TAG -o run -- python bench_fk.py --cpu-seconds 1 > /dev/null 2> $O/prof_fk_$TAG.err || exit 5
head -12 $O/prof_fk_$TAG/run_kernel_stats.csv | cut -c1-160
