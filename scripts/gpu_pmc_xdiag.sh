#!/bin/bash
# Where the xgemm kernels' waves spend their cycles (single stream): SQ wait /
# active shares, MFMA busy, LDS activity and bank conflicts, VALU / MFMA instructions
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp TIK_SPLIT=0
OUT=gpurun_out; TAG=${1:-xdiag}; mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compare --no-profile"
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmcx1_$TAG -o run -- $B > /dev/null 2> $OUT/pmcx1_$TAG.err || exit $?
python scripts/pmc_generic.py $OUT/pmcx1_$TAG xgemm > $OUT/pmcx_$TAG.txt
timeout -k 10 60 rocprofv3 --list-avail > $OUT/pmc_avail.txt 2>&1 || true
C2=""
for c in SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES; do
  grep -q "\b$c\b" $OUT/pmc_avail.txt && C2="$C2 $c"
done
C2=$(echo $C2 | cut -d' ' -f1-7)
echo "pass 2 counters: $C2"
if [ -n "$C2" ]; then
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $C2 GRBM_GUI_ACTIVE -d $OUT/pmcx2_$TAG -o run -- $B > /dev/null 2> $OUT/pmcx2_$TAG.err || exit $?
  python scripts/pmc_generic.py $OUT/pmcx2_$TAG xgemm >> $OUT/pmcx_$TAG.txt
fi
cat $OUT/pmcx_$TAG.txt
