#!/bin/bash
# r06 warm: does the untimed warmup length change the timed step? (same box, fresh process each)
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2; do
  for w in 5 30 100; do
    timeout -k 10 120 python bench.py --steps 20 --warmup $w --no-profile --no-cpu-baseline --no-compare --no-extras > $O/bench_r06w.json 2> $O/bench_r06w.err || exit 1
    python -c "import json;d=json.load(open('$O/bench_r06w.json'));print('warmup $w steps 20', d['ms_per_step'])"
  done
  timeout -k 10 120 python bench.py --steps 100 --warmup 30 --no-profile --no-cpu-baseline --no-compare --no-extras > $O/bench_r06w.json 2> $O/bench_r06w.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_r06w.json'));print('warmup 30 steps 100', d['ms_per_step'])"
done | tee $O/ab_r06warm.txt
