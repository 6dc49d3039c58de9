#!/bin/bash
# r04: HIP API + memory-copy + kernel trace of the 100-pair sweep (where the
# host stalls the GPU between batches); no counters in this run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/ht_sweep -o run -- python3 tools/bench_sweep.py --pairs 100 --reps 1 > gpurun_out/ht_sweep.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/ht_sweep.log; exit 1; }
ls -la gpurun_out/ht_sweep
echo done
