# TG epilogue change: IK parity suite, TG phase trace, headline bench (2 runs)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TIK_TG_TRACE=1 TIK_SPLIT=0 timeout -k 10 300 python scripts/stb_trace.py > $O/tg_trace.txt 2>&1 || exit $?
grep "^TG" $O/tg_trace.txt | tail -3
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-profile --steps 40 > $O/b.json 2> $O/b.err || exit $?
cat $O/b.json
done
