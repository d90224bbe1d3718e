set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-x}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -4 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']);print({k:v['avg_ms'] for k,v in d['forward']['launches'].items()});print(d.get('other_precision'))"
timeout -k 10 300 python bench_stream.py --frames 3000 > $OUT/stream_$TAG.json 2> $OUT/stream_$TAG.err; rc=$?; cat $OUT/stream_$TAG.json; tail -2 $OUT/stream_$TAG.err; echo "stream rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_stream.py --frames 1000 --no-graph > $OUT/stream_eager_$TAG.json 2>&1; cat $OUT/stream_eager_$TAG.json
