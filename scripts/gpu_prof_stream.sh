set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-ps}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stream_$TAG -o run -- python bench_stream.py --frames 300 --warmup 20 --no-graph > $OUT/prof_stream_$TAG.json 2> $OUT/prof_stream_$TAG.err; echo rc=$?
f=$(find $OUT/prof_stream_$TAG -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-8 | head -30
