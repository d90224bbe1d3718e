#!/bin/bash
# Same-box A/B of the nontemporal layer-output stores on the final build
# (runtime flag XArgs::nts): all layers (default), none (TIK_XNTS=0), layers 2-7 only (252)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ROUNDS=3 bash scripts/gpu_ab_libs.sh nts new new:TIK_XNTS=0 new:TIK_XNTS=252 || exit 1
