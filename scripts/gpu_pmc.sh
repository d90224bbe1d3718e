# PMC passes on the bench (each counter group in its own run; kernel-trace only, no sys/runtime trace)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-pmc}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-compare > $OUT/bench_$TAG.json 2>$OUT/bench_$TAG.err || exit $?
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $OUT/pmc_${TAG}_$i -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare > /dev/null 2> $OUT/pmc_${TAG}_$i.err; rc=$?
  echo "pass $i ($ctr) rc=$rc"
  [ $rc -eq 0 ] || break
done
cat $OUT/bench_$TAG.json
