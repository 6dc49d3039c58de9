#!/bin/bash
# r04: LLVM scheduler variants of the STOI translation unit (4,096 10-s cells,
# tools/bench_stoi.py, alternating), then the STOI tests of the fastest
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  REPS=5 bash tools/ab_stoi.sh libcse.so libcse_smclause.so libcse_smaxilp.so libcse_strackers.so || exit 1
done
echo done
