#!/bin/bash
# r06 k: XTWG with z stored during the next tile's T K block 0 (parity + same-box A/B + bench)
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "xtws or golden or batch_invariant or xgraph" > $O/pytest_r06k.log 2>&1 || { tail -30 $O/pytest_r06k.log; exit 1; }
tail -2 $O/pytest_r06k.log
for i in 1 2; do
  for v in old new; do echo "== $v"; timeout -k 10 60 ./build/xwbench_$v 1024 32 20 | grep -E "XTW|tune   0|tune  64" || exit 1; done
done > $O/xwbench_r06k.txt 2>&1
cat $O/xwbench_r06k.txt
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-compare --no-extras > $O/bench_r06k.json 2> $O/bench_r06k.err || exit 1
python -c "import json;d=json.load(open('$O/bench_r06k.json'));print(d['ms_per_step'], d['forward']['launches'].get('XTWG.L3'), d['forward']['launches'].get('XTWG.L4'))"
