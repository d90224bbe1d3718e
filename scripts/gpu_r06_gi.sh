#!/bin/bash
# r06 gi: XTWG gcn-phase split units read one item ahead and interleaved into the next item's MFMAs, vs r06_w, same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_gi.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "golden or batch_invariant or xtws" > $O/pytest_r06gi.log 2>&1 || { tail -20 $O/pytest_r06gi.log; exit 1; }
tail -1 $O/pytest_r06gi.log
for i in 1 2 3; do
  for v in base gi; do
    TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_$v.so timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06gi.json 2> $O/bench_r06gi.err || exit 1
    python -c "
import json;d=json.load(open('$O/bench_r06gi.json'));L=d['forward']['launches']
print('%-6s' % '$v', d['ms_per_step'], ' '.join('%s %.4f' % (k, v['avg_ms']) for k, v in L.items() if k.startswith(('XTW','XT1'))))"
  done
done | tee $O/ab_r06gi.txt
