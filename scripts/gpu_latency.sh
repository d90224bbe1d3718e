# online-IK latency: the default small-batch path vs the DMA path forced (TIK_GEMM_PATH=dma),
# per-kernel durations of the B=1 step, and the TG phase trace at the bench size
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 300 python bench_stream.py --frames 2000 > $O/def.json 2> $O/def.err || exit $?
echo "default $(cat $O/def.json)"
TIK_GEMM_PATH=dma timeout -k 10 300 python bench_stream.py --frames 2000 > $O/dma.json 2> $O/dma.err || exit $?
echo "dma $(cat $O/dma.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_def -o run -- python bench_stream.py --frames 300 --no-graph > /dev/null 2> $O/prof_def.err || exit $?
TIK_GEMM_PATH=dma timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dma -o run -- python bench_stream.py --frames 300 --no-graph > /dev/null 2> $O/prof_dma.err || exit $?
TIK_TG_TRACE=1 TIK_SPLIT=0 timeout -k 10 300 python scripts/stb_trace.py > $O/tg_trace.txt 2>&1 || exit $?
tail -8 $O/tg_trace.txt
