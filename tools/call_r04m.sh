#!/bin/bash
# r04: LLVM scheduler variants of the n_fft 512 translation unit (13-pair
# A/B, alternating): the product build, max-memory-clause, AMDGPU RP trackers
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  STEPS=5 bash tools/ab_libs.sh libcse.so libcse_mclause.so libcse_trackers.so || exit 1
done
echo done
