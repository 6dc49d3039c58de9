#!/bin/bash
# r04: the packed 512 frame without the gain stage's s_setprio(1) (13 pairs,
# three alternating rounds against the product)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  STEPS=5 bash tools/ab_libs.sh libcse.so libcse_np.so || exit 1
done
echo done
