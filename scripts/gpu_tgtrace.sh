set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/tgt; mkdir -p $O
TIK_TG_TRACE=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compare > $O/t.json 2> $O/t.err || exit $?
grep "TG L" $O/t.err | tail -3
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved'],d['roofline']['frac']);print({k:v['avg_ms'] for k,v in d['forward']['launches'].items()})"
