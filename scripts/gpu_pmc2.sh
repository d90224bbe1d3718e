set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-pmc2}
mkdir -p $OUT
python -m temporal_inverse_kinematics_amd._build > $OUT/build.log 2>&1 || exit 2
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d $OUT/pmc_${TAG}_$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compare --precision ${PREC:-f16x3} > /dev/null 2> $OUT/pmc_${TAG}_$i.err; rc=$?
  echo "pass $i ($ctr) rc=$rc"; tail -2 $OUT/pmc_${TAG}_$i.err
  [ $rc -eq 0 ] || break
done
