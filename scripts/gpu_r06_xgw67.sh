#!/bin/bash
# r06 xgw67: the gcn of layers 6 / 7 on the tiled XG128 (TIK_XGW=63) vs xgraph (default), same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2 3; do
  for m in 255 63 127 191; do
    TIK_XGW=$m timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06x67.json 2> $O/bench_r06x67.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06x67.json'));L=d['forward']['launches']
print('xgw %-4s' % '$m', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.endswith(('L6','L7'))))"
  done
done | tee $O/ab_r06xgw67.txt
