#!/bin/bash
# r06 xg: same-box A/B of xgraph setprio for waves 4-7 (build/ab/libtik_xg{0,1}.so)
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2 3; do
  for v in 0 1; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_xg$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06xg_$v.json 2> $O/bench_r06xg_$v.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06xg_$v.json'));L=d['forward']['launches']
print('$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, L[k]['avg_ms']) for k in ('XGW.L2','XGW.L3','XGW.L6','XGW.L7')))"
  done
done | tee $O/ab_r06xg.txt
