# IK step time vs the number of concurrent parts (streams) of a split batch
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/splitn; mkdir -p $O
for n in 2 3 4 2 3 4; do
  TIK_SPLIT_N=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-compare --no-profile --steps 40 > $O/n$n.json 2> $O/n$n.err || exit $?
  python -c "import json;d=json.load(open('$O/n$n.json'));print('split_n=$n', d['value'], d['ms_per_step'])"
done
