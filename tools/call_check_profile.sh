#!/bin/bash
# One round-checkpoint GPU call: the fp64 matrix/vector micro-benchmark, the
# -m gpu suite + smoke + bench line (tools/gpu_check.sh), then every kernel
# trace and PMC pass (tools/profile_all.sh TAG).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -x tools/micro/mfma_f64 ]; then
  timeout -k 10 60 tools/micro/mfma_f64 > gpurun_out/mfma_f64.txt 2>&1 || exit 1
  cat gpurun_out/mfma_f64.txt
fi
bash tools/gpu_check.sh && bash tools/profile_all.sh ${TAG:-r03d}
