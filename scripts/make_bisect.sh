#!/bin/bash
# Builds the three bisection trees of scripts/gpu_bisect.sh under bisect/ (git-ignored)
set -eu
cd "$(dirname "$0")/.."
rm -rf bisect; mkdir -p bisect
for v in v0 v1 v2; do mkdir -p bisect/$v; git archive 283cbfa | tar -x -C bisect/$v; done
git diff 283cbfa d503083 -- temporal_inverse_kinematics_amd/csrc/layer0.hip temporal_inverse_kinematics_amd/csrc/cgemm3.hip | (cd bisect/v1 && patch -p1)
git diff 283cbfa d503083 -- temporal_inverse_kinematics_amd/csrc/tgemm.hip | (cd bisect/v2 && patch -p1)
for v in v1 v2; do printf '\n#ifndef TIK_FENCE_BEGIN\n#define TIK_FENCE_BEGIN() ((void)0)\n#define TIK_FENCE_END() ((void)0)\n#endif\n' >> bisect/$v/temporal_inverse_kinematics_amd/csrc/cgemm3_dev.h; done
for v in v0 v1 v2; do cp scripts/diag_streams.py scripts/diag_mproc.py bisect/$v/scripts/; (cd bisect/$v && python -m temporal_inverse_kinematics_amd._build > build.log 2>&1); done
for v in v0 v1 v2; do rm -rf bisect/$v/tests/golden bisect/$v/profiles bisect/$v/temporal_inverse_kinematics_amd/build; done
