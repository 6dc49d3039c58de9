#!/bin/bash
# r04: step vs kernel time at the per-GPU share of an 8-GPU strong-scaling run
# (13 pairs per GPU), 10 timed steps; then a kernel trace of the same run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 13 13 100; do
  PAIRS=$p STEPS=10 bash tools/ab_libs.sh libcse.so || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_r04l -o run -- python3 bench.py --pairs 13 --steps 6 --warmup 2 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep > gpurun_out/kt_r04l.log 2>&1 || { echo "kt failed"; tail -5 gpurun_out/kt_r04l.log; exit 1; }
echo done
