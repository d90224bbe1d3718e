set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/evt; mkdir -p $O
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-profile --steps 40 > $O/np.json 2> $O/e.err || exit $?; cat $O/np.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 40 > $O/p.json 2> $O/e.err || exit $?; python -c "import json;d=json.load(open('$O/p.json'));print(d['value'],d['ms_per_step'])"
done
