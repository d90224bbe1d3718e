# PMC passes over the kernel tuning harness (one counter group per pass, kernel-trace only)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-kb}
mkdir -p $OUT
i=0
for ctr in "FETCH_SIZE" "TCC_HIT_sum" "TCC_MISS_sum" "SQ_WAIT_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES" "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $OUT/pmc_${TAG}_$i -o run -- ./build/kbench 1024 64 2 > $OUT/pmc_${TAG}_$i.log 2>&1; rc=$?
  echo "pass $i ($ctr) rc=$rc"
  [ $rc -eq 0 ] || break
done
