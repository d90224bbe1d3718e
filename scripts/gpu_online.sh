# online IK step: graph vs eager, kernel time under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/online; mkdir -p $O
timeout -k 10 120 python bench_stream.py --frames 2000 > $O/graph.json 2> $O/graph.err || exit $?
python -c "import json;d=json.load(open('$O/graph.json'));print('graph', d['value'], d['p99_us'])"
timeout -k 10 120 python bench_stream.py --frames 2000 --no-graph > $O/eager.json 2> $O/eager.err || exit $?
python -c "import json;d=json.load(open('$O/eager.json'));print('eager', d['value'], d['p99_us'])"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench_stream.py --frames 1000 > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-7
