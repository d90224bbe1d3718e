#!/bin/bash
# Builds the bisection trees of scripts/gpu_bisect.sh under bisect/ (git-ignored):
# the pre-fix tree 283cbfa, plus subsets of the fix commit d503083's kernel changes:
#   v0 as it was; v1 mix constants in registers in gcn0 AND the cgemm3 graph epilogue;
#   v2 only the readfirstlane DMA soffset in tgemm (no waterfall loops);
#   v3 only gcn0's mix constants in registers; v4 only cgemm3's.
set -eu
cd "$(dirname "$0")/.."
rm -rf bisect; mkdir -p bisect
for v in v0 v1 v2 v3 v4; do mkdir -p bisect/$v; git archive 283cbfa | tar -x -C bisect/$v; done
K=temporal_inverse_kinematics_amd/csrc
git diff 283cbfa d503083 -- $K/layer0.hip $K/cgemm3.hip | (cd bisect/v1 && patch -p1)
git diff 283cbfa d503083 -- $K/tgemm.hip | (cd bisect/v2 && patch -p1)
git diff 283cbfa d503083 -- $K/layer0.hip | (cd bisect/v3 && patch -p1)
git diff 283cbfa d503083 -- $K/cgemm3.hip | (cd bisect/v4 && patch -p1)
for v in v1 v2 v3 v4; do printf '\n#ifndef TIK_FENCE_BEGIN\n#define TIK_FENCE_BEGIN() ((void)0)\n#define TIK_FENCE_END() ((void)0)\n#endif\n' >> bisect/$v/$K/cgemm3_dev.h; done
for v in v0 v1 v2 v3 v4; do
  cp scripts/diag_streams.py scripts/diag_mproc.py bisect/$v/scripts/
  (cd bisect/$v && python -m temporal_inverse_kinematics_amd._build > build.log 2>&1)
  rm -rf bisect/$v/tests/golden bisect/$v/profiles bisect/$v/temporal_inverse_kinematics_amd/build
done
