#!/bin/bash
# r06 nt2: nontemporal xgraph row loads (xgnt: every layer, xgnt1: one-pass layers only) vs r06_v on the
# IK step; nontemporal blend-GEMM output stores (bnt) vs r06_v on the FK step; same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xgnt.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "golden or batch_invariant" > $O/pytest_r06nt2.log 2>&1 || { tail -20 $O/pytest_r06nt2.log; exit 1; }
tail -1 $O/pytest_r06nt2.log
for i in 1 2 3; do
  for v in base xgnt xgnt1; do
    L=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so; [ $v = base ] && L=$GRAFT_REPO_ROOT/temporal_inverse_kinematics_amd/libtik.so
    TIK_LIB=$L timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06nt2.json 2> $O/bench_r06nt2.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06nt2.json'));L=d['forward']['launches']
print('%-6s' % '$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith('XGW')))"
  done
done | tee $O/ab_r06nt2_ik.txt
run() {
  timeout -k 10 120 python -c "
import json, bench_fk; d = bench_fk.measure_fk(4096, 10, 20)
print('$1', d['ms_per_step'], d['value'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))"
}
for i in 1 2 3; do
  run base || exit 1
  TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_bnt.so run bnt || exit 1
done | tee $O/ab_r06nt2_fk.txt
