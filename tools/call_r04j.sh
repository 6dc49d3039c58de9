#!/bin/bash
# r04: where a 100-pair sweep's GPU time goes (kernel trace of tools/bench_sweep.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_sweep100 -o run -- python3 tools/bench_sweep.py --pairs 100 --reps 1 > gpurun_out/kt_sweep100.log 2>&1 || { echo "kt failed"; tail -5 gpurun_out/kt_sweep100.log; exit 1; }
tail -2 gpurun_out/kt_sweep100.log
echo done
