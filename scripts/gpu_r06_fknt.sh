#!/bin/bash
# r06 fknt: sparse skinning with nontemporal vertex stores (nt), v_posed loads (ntl), both (ntb) vs r06_w, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_ntb.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fk.py > $O/pytest_r06fknt.log 2>&1 || { tail -20 $O/pytest_r06fknt.log; exit 1; }
tail -1 $O/pytest_r06fknt.log
run() {
  timeout -k 10 120 python -c "
import json, bench_fk; d = bench_fk.measure_fk(4096, 10, 20)
print('$1', d['ms_per_step'], d['value'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
}
for i in 1 2 3; do
  run "base" || exit 1
  for v in nt ntl ntb; do TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so run "$v" || exit 1; done
done | tee $O/ab_r06fknt.txt
