#!/bin/bash
# r06 fklmk: landmarks per chunk in the chunk's stream + skinning workgroups per CU, vs the r06 tree, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fk.py > $O/pytest_r06fkl.log 2>&1 || { tail -20 $O/pytest_r06fkl.log; exit 1; }
tail -1 $O/pytest_r06fkl.log
run() {
  timeout -k 10 120 python -c "
import json, bench_fk; d = bench_fk.measure_fk(4096, 10, 20)
print('$1', d['ms_per_step'], d['value'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
}
for i in 1 2 3; do
  TIK_FK_WPC=4 TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_base.so run "base wpc4" || exit 1
  TIK_FK_WPC=4 run "lmk wpc4" || exit 1
  run "lmk wpc8" || exit 1
  TIK_FK_WPC=16 run "lmk wpc16" || exit 1
done | tee $O/ab_r06fklmk.txt
