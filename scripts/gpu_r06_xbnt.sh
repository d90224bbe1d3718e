#!/bin/bash
# r06 xbnt: block 1's x-image LDS-DMA with the nt cache policy vs r06_u, IK step, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xbnt.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "golden or batch_invariant or xblock" > $O/pytest_r06xbnt.log 2>&1 || { tail -20 $O/pytest_r06xbnt.log; exit 1; }
tail -1 $O/pytest_r06xbnt.log
for i in 1 2 3 4; do
  for v in base xbnt; do
    L=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so; [ $v = base ] && L=$GRAFT_REPO_ROOT/temporal_inverse_kinematics_amd/libtik.so
    TIK_LIB=$L timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06xbnt.json 2> $O/bench_r06xbnt.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06xbnt.json'));L=d['forward']['launches']
print('%-6s' % '$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith('XB')))"
  done
done | tee $O/ab_r06xbnt.txt
