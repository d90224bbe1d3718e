#!/bin/bash
# r06 fkwpc: sparse skinning workgroups per CU (TIK_FK_WPC; default 4) and diagnostic builds
# (TIK_FK_DIAG 1: every lane reads the same joints, no LDS bank conflicts; 2: no vertex stores;
# 3: no v_posed loads), same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
run() {
  timeout -k 10 120 python -c "
import json, bench_fk; d = bench_fk.measure_fk(4096, 10, 20)
print('$1', d['ms_per_step'], d['value'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
}
for i in 1 2; do
  for w in 4 2 3 8; do TIK_FK_WPC=$w run "wpc $w" || exit 1; done
  for d in 1 2 3; do TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_fkd$d.so run "diag $d" || exit 1; done
done | tee $O/ab_r06fkwpc.txt
