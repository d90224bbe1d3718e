#!/bin/bash
# r06 nomix: what the VALU graph mix costs in XB0 / XB1 (diagnostic build with only the diagonal mix term; results wrong by design)
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for v in base nomix; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06nm.json 2> $O/bench_r06nm.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06nm.json'));L=d['forward']['launches']
print('$v', d['ms_per_step'], 'XB0 %.4f XB1 %.4f' % (L['XB0.L0']['avg_ms'], L['XB1.L1']['avg_ms']))"
  done
done | tee $O/ab_r06nomix.txt
