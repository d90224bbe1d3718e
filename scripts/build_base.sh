#!/bin/bash
# Build libtik.so of git revision $1 (default HEAD) into ab/libtik_base.so, for
# same-box A/B runs (TIK_LIB selects the library): box-to-box variance (~5 %)
# is larger than most single-kernel changes.
set -eu
REV=${1:-HEAD}
cd "$(dirname "$0")/.."
WT=/tmp/tik_wt_base
git worktree remove --force $WT 2>/dev/null || true
git worktree add -f --detach $WT $REV > /dev/null
(cd $WT && python -m temporal_inverse_kinematics_amd._build > /dev/null)
mkdir -p ab
cp $WT/temporal_inverse_kinematics_amd/libtik.so ab/libtik_base.so
git worktree remove --force $WT
echo "ab/libtik_base.so <- $(git rev-parse --short $REV)"
