#!/bin/bash
# Does any kernel write into another workgroup's LDS? scripts/lds_victim
# (per-lane or broadcast re-reads of an LDS pattern) runs while 3 processes run
# the IK forward of a tree (the pre-fix bisect/v0, or this tree), and counts words
# that changed. Build: hipcc --offload-arch=gfx950 -O3 scripts/lds_victim.hip -o scripts/bin/lds_victim
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/victim; mkdir -p $O
for tree in ${TREES:-bisect/v0 .}; do for mode in ${MODES:-0 1}; do
  tag=$(basename $(cd $tree && pwd))_m$mode
  timeout -k 10 60 ./scripts/bin/lds_victim 20 $mode > $O/victim_$tag.json 2>&1 &
  vp=$!
  pids=""
  for k in 1 2 3; do (cd $tree && AGG_SECONDS=20 timeout -k 10 60 python scripts/diag_mproc.py child > $O/agg_${tag}_$k.txt 2>&1) & pids="$pids $!"; done
  wait $vp; vrc=$?
  for p in $pids; do wait $p; done
  echo "$tree mode $mode (rc $vrc): victim $(cat $O/victim_$tag.json | tr '\n' ' ') aggressors worst: $(cat $O/agg_${tag}_*.txt | grep -v amdgpu | tr '\n' ' ')"
  [ $vrc -eq 0 ] || exit $vrc
done; done
