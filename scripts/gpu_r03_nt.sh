#!/bin/bash
# Same-box A/B of two xgemm builds against the default in-tree one, on the IK
# bench (parity first) and the FK bench (FK parity first):
#   nt   ab/libtik_nt.so,   TIK_HIPCC_FLAGS=-DTIK_XNT      (nontemporal epilogue stores)
#   prio ab/libtik_prio.so, TIK_HIPCC_FLAGS=-DTIK_XPRIO=3  (epilogue wave priority)
# plus the default build with the batch split into 3 / 4 parts (TIK_SPLIT_N),
# and on FK the 12-row skinning layout (s12: TIK_FK_SKIN12=1; parity tests first).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab_nt; mkdir -p $O
TIK_FK_SKIN12=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fk.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_fk_new.log 2>&1; rc=$?
echo "pytest fk s12: $(tail -1 $O/pt_fk_new.log)"; [ $rc -eq 0 ] || exit 2
TIK_LIB=ab/libtik_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fk.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_fk.log 2>&1; rc=$?
echo "pytest fk nt: $(tail -1 $O/pt_fk.log)"; [ $rc -eq 0 ] || exit 2
for r in 1 2 3; do for v in new s12 nt prio; do
  L=""; E="TIK_AB=1"
  case $v in s12) E=TIK_FK_SKIN12=1;; nt|prio) L=ab/libtik_$v.so;; esac
  env $E TIK_LIB=$L timeout -k 10 200 python bench_fk.py --cpu-seconds 1 > $O/fk_$v$r.json 2> $O/fk_$v$r.err || exit 3
  python -c "import json;d=json.load(open('$O/fk_$v$r.json'));print('fk $v$r', d['value'], d['ms_per_step'], d['gemm_tflops'])"
done; done
AB_TESTS=1 ROUNDS=0 bash scripts/gpu_ab_libs.sh nt nt prio || exit 1
ROUNDS=3 bash scripts/gpu_ab_libs.sh nt new nt prio new:TIK_SPLIT_N=3 new:TIK_SPLIT_N=4 || exit 1
