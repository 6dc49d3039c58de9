#!/bin/bash
# Round-end GPU call: the -m gpu suite + smoke + bench line (tools/gpu_check.sh),
# an A/B of the analysis stream layout (tools/ab_hops.sh), then every kernel
# trace and PMC pass of the final kernels (tools/profile_all.sh TAG).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
VARS="1 0 1 0" bash tools/ab_hops.sh > gpurun_out/ab_hops.txt 2>&1 || exit 1
cat gpurun_out/ab_hops.txt
bash tools/profile_all.sh ${TAG:-r03e}
