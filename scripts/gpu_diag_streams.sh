set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dstreams7; mkdir -p $O
timeout -k 10 120 python scripts/diag_streams.py 4 12 > $O/s4.json 2> $O/s4.err || exit $?; cat $O/s4.json
timeout -k 10 240 python scripts/diag_mproc.py 4 > $O/mp.json 2> $O/mp.err || exit $?; cat $O/mp.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved']);print({k:v['avg_ms'] for k,v in d['forward']['launches'].items()})"
