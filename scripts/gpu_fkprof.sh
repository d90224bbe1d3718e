# per-kernel timing of the FK+LBS step (config #4)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/fkprof; mkdir -p $O
TAG=${1:-x}
timeout -k 10 200 python bench_fk.py --cpu-seconds 0.5 > $O/fk_$TAG.json 2> $O/fk_$TAG.err || exit $?
cat $O/fk_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python bench_fk.py --cpu-seconds 0.5 > /dev/null 2> $O/prof_$TAG.err || exit $?
python scripts/prof_summary.py $O/prof_$TAG 2>/dev/null | head -20 || find $O/prof_$TAG -name "*stats*" | head
