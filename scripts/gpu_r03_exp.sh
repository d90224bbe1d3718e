#!/bin/bash
# xgemm experiments: per-launch times with parts switched off (TIK_XTUNE bits), then PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${1:-r03_exp}; mkdir -p $OUT
for t in 0 1 2 3 4 8 7; do
  TIK_XTUNE=$t timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-compare --no-cpu-baseline > $OUT/exp_${TAG}_$t.json 2>/dev/null || exit 3
  python -c "
import json; d=json.load(open('$OUT/exp_${TAG}_$t.json'))
print('tune $t', ' '.join(f\"{k}={v['avg_ms']:.3f}\" for k,v in d['forward']['launches'].items() if k.startswith('X')))
"
done
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare --no-profile"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/pmc1_$TAG -o run -- $B > /dev/null 2> $OUT/pmc1_$TAG.err || exit 4
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_SALU -d $OUT/pmc2_$TAG -o run -- $B > /dev/null 2> $OUT/pmc2_$TAG.err || exit 5
echo done
