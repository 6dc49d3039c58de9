#!/bin/bash
# Round-end GPU call: the -m gpu suite + smoke + bench line (tools/gpu_check.sh),
# then every kernel trace and PMC pass of the final kernels
# (tools/profile_all.sh TAG).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
bash tools/profile_all.sh ${TAG:-r03e}
