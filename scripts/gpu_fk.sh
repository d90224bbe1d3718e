set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m temporal_inverse_kinematics_amd._build > gpurun_out/build.log 2>&1 || exit 2
timeout -k 10 600 python -m pytest tests/test_gpu_fk.py -q -x > gpurun_out/pytest_fk.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_fk.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench_fk.py > gpurun_out/bench_fk.json 2> gpurun_out/bench_fk.err; rc=$?
cat gpurun_out/bench_fk.json; tail -3 gpurun_out/bench_fk.err; echo "bench rc=$rc"
