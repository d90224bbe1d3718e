# A/B of an env toggle on the headline bench, interleaved in one process-per-run sequence on one box
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab; mkdir -p $O
VAR=${1:-TIK_SPLIT}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ik.py -x -q --timeout 300 > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --no-profile --steps 40 > $O/b.json 2> $O/b.err || exit $?
  echo "$VAR=$v $(cat $O/b.json)"
done; done
