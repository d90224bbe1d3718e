# PMC passes + rocprofv3 kernel stats of the bench, all SINGLE-STREAM
# (--no-extras: the FK and online extras would add same-symbol xgemm launches, the FK blend GEMM, to the per-kernel PMC averages)
# (TIK_SPLIT=0): with the two-stream split half the dispatches are half-batch
# launches, and per-dispatch averages would mix the two sizes. Separate passes
# (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE), kernel
# trace only. Usage: bash scripts/gpu_pmc_all.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp TIK_SPLIT=0
OUT=gpurun_out
TAG=${1:-pmc}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o run -- $B > /dev/null 2> $OUT/pmc_fetch_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o run -- $B > /dev/null 2> $OUT/pmc_write_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_mfma_$TAG -o run -- $B > /dev/null 2> $OUT/pmc_mfma_$TAG.err || exit $?
python scripts/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG $OUT/pmc_traffic_$TAG.json > $OUT/pmc_traffic_$TAG.txt 2>&1
python scripts/pmc_mfma.py $OUT/pmc_mfma_$TAG $OUT/pmc_mfma_$TAG.json > $OUT/pmc_mfma_$TAG.txt 2>&1
cat $OUT/pmc_traffic_$TAG.txt $OUT/pmc_mfma_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-compare --no-extras > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || exit $?
echo "pmc + stats done"
