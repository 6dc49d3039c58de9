#!/bin/bash
# r04: the 100-pair sweep after the host bookkeeping changes (two runs), then
# the HIP API trace of one more for the prologue / epilogue between syncs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_sweep.py --pairs 100 --reps 2 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/ht_sweep2 -o run -- python3 tools/bench_sweep.py --pairs 100 --reps 1 > gpurun_out/ht_sweep2.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/ht_sweep2.log; exit 1; }
echo done
