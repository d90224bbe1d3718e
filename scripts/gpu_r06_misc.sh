#!/bin/bash
# Round 6: full GPU suite + smoke, then same-box A/Bs: the two-part split
# (TIK_SPLIT=0 vs default) and the online step (hipGraph replay vs eager launch).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-misc}; mkdir -p $OUT
bash scripts/gpu_tests.sh $TAG || exit $?
i=0
for cfg in "TIK_SPLIT=0" "-" "TIK_SPLIT=0" "-"; do
  i=$((i + 1))
  envs=""; [ "$cfg" = "-" ] || envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-extras --no-profile --steps 30 > $OUT/absplit_${TAG}_$i.json 2> $OUT/absplit_${TAG}_$i.err || exit $?
  python -c "import json;d=json.load(open('$OUT/absplit_${TAG}_$i.json'));print('$cfg', d['value'], d['ms_per_step'])"
done
for g in "" "--no-graph" "" "--no-graph"; do
  timeout -k 10 200 python bench_stream.py --frames 3000 $g > $OUT/abstream_${TAG}.json 2>> $OUT/abstream_${TAG}.err || exit $?
  python -c "import json;d=json.load(open('$OUT/abstream_${TAG}.json'));print('online $g', d.get('value'), d.get('p99_us'))"
done
