#!/bin/bash
# r06 xpt: XT128 on the persistent xgemm_pt kernel (build/ab/libtik_xpt.so, -DTIK_XPT128=1) vs the tiled default, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xpt.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "golden or batch_invariant" > $O/pytest_r06xpt.log 2>&1 || { tail -20 $O/pytest_r06xpt.log; exit 1; }
tail -1 $O/pytest_r06xpt.log
for i in 1 2; do
  for v in base xpt; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06xpt.json 2> $O/bench_r06xpt.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06xpt.json'));L=d['forward']['launches']
print('$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith(('XT128', 'XP128'))))"
  done
done | tee $O/ab_r06xpt.txt
