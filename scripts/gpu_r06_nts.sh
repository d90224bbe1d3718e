#!/bin/bash
# r06 nts: nontemporal vs plain layer-output stores (TIK_NTS_MASK builds: bit 0 XGW, bit 1 xtws, bit 2 XT128; 7 = default), same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for v in 7 0 3 5 6; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_nts$v.so timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06nts.json 2> $O/bench_r06nts.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06nts.json'));L=d['forward']['launches']
print('mask $v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith(('XGW','XT128','XTWG'))))"
  done
done | tee $O/ab_r06nts.txt
