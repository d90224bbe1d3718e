#!/bin/bash
# r06 nt3: nontemporal row loads in xgraph (xgnt) and in xgraph + xtws (xgtw) vs r06_v, IK step, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xgtw.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "golden or batch_invariant or xtws" > $O/pytest_r06nt3.log 2>&1 || { tail -20 $O/pytest_r06nt3.log; exit 1; }
tail -1 $O/pytest_r06nt3.log
for i in 1 2 3 4; do
  for v in base xgnt xgtw; do
    L=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so; [ $v = base ] && L=$GRAFT_REPO_ROOT/temporal_inverse_kinematics_amd/libtik.so
    TIK_LIB=$L timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06nt3.json 2> $O/bench_r06nt3.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06nt3.json'));L=d['forward']['launches']
print('%-6s' % '$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith(('XGW','XTWG'))))"
  done
done | tee $O/ab_r06nt3.txt
