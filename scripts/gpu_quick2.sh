set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/q2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 300 > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved'],d['roofline']['frac']);print({k:v['avg_ms'] for k,v in d['forward']['launches'].items()})"
