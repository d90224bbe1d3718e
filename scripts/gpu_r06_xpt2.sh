#!/bin/bash
# r06 xpt2: tiled XT128 vs persistent XP128, each with and without its epilogue row stores (diagnostic builds; no-store results are wrong by design)
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for v in base xtns xpt xptns; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06xpt.json 2> $O/bench_r06xpt.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06xpt.json'));L=d['forward']['launches']
print('%-6s' % '$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith(('XT128', 'XP128'))))"
  done
done | tee $O/ab_r06xpt2.txt
