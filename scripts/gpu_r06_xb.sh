#!/bin/bash
# r06 xb: same-box A/B of block 0/1 variants (TIK_XB_DMAPRE x TIK_XB_PRIO builds in build/ab), parity on the default
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "xblock or golden or batch_invariant" > $O/pytest_r06xb.log 2>&1 || { tail -30 $O/pytest_r06xb.log; exit 1; }
tail -2 $O/pytest_r06xb.log
for i in 1 2; do
  for v in 00 10 01 11; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xb$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06xb_$v.json 2> $O/bench_r06xb_$v.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06xb_$v.json'));L=d['forward']['launches']
print('$v', d['ms_per_step'], 'XB0 %.4f XB1 %.4f' % (L['XB0.L0']['avg_ms'], L['XB1.L1']['avg_ms']))"
  done
done | tee $O/ab_r06xb.txt
