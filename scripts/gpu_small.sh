# small-batch change: GPU parity suite, then online-IK latency and the headline bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/small; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_stream.py --frames 3000 > $O/stream.json 2> $O/stream.err || exit $?
cat $O/stream.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-profile --steps 40 > $O/b.json 2> $O/b.err || exit $?
cat $O/b.json
