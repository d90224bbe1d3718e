# PMC passes over the kernel tuning harness, one layer (default L3), one counter group per pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-kb}; LAYER=${2:-3}
mkdir -p $OUT
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" "TA_BUSY_avr TA_TA_BUSY_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $OUT/pmc_${TAG}_$i -o run -- ./build/kbench 1024 64 2 $LAYER > $OUT/pmc_${TAG}_$i.log 2>&1; rc=$?
  echo "pass $i ($ctr) rc=$rc"
done
exit 0
