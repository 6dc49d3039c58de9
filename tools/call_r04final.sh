#!/bin/bash
# r04 round-end evidence from one box: the -m gpu suite + smoke + bench line
# (tools/gpu_check.sh), then every kernel trace and PMC pass of the final
# kernels (tools/profile_all.sh TAG), then the bench line again so it carries
# nothing stale.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit $?
bash tools/profile_all.sh ${TAG:-r04f} || exit $?
echo done
