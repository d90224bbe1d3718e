# quick iteration: IK parity tests + bench (no CPU baseline / second precision)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-q}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
timeout -k 10 600 python -m pytest tests/test_gpu_ik.py -q -x > $OUT/pytest_ik_$TAG.log 2>&1; rc=$?
tail -3 $OUT/pytest_ik_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved']);print({k:v['avg_ms'] for k,v in d['forward']['launches'].items()})"
