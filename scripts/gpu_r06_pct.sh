#!/bin/bash
# r06 pct: two-part split with unequal parts (TIK_SPLIT_PCT = part 0's share), same box
cd $GRAFT_REPO_ROOT
O=gpurun_out
export TIK_LIB=$GRAFT_REPO_ROOT/build/ab/libtik_pct.so
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ik.py -k "batch_invariant or split or stream" > $O/pytest_r06pct.log 2>&1 || { tail -20 $O/pytest_r06pct.log; exit 1; }
tail -1 $O/pytest_r06pct.log
for i in 1 2; do
  for p in 50 40 60 30 70; do
    TIK_SPLIT_PCT=$p timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-profile --no-cpu-baseline --no-compare --no-extras > $O/bench_r06pct.json 2> $O/bench_r06pct.err || exit 1
    python -c "import json;d=json.load(open('$O/bench_r06pct.json'));print('pct $p', d['ms_per_step'])"
  done
done | tee $O/ab_r06pct.txt
