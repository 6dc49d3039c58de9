#!/bin/bash
# r06 profiling call: kernel traces and PMC passes of the product build
# (tools/profile_all.sh, each pass its own rocprofv3 run) plus the shader
# clock over a 20-pair sweep and over a solo STOI run (tools/clock_trace.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06a}
WHAT=${WHAT:-kt512 pmc512 pmcpk pmc512s kt1024 pmc1024 pmcpk1024}
bash tools/profile_all.sh $TAG $WHAT || exit $?
if [ -n "$CLOCKS" ]; then
  timeout -k 10 240 python3 tools/clock_trace.py gpurun_out/clock_sweep.json -- python3 tools/bench_sweep.py --pairs 20 --reps 1 > gpurun_out/clock_sweep.log 2>&1 || { echo "clock sweep failed"; tail -5 gpurun_out/clock_sweep.log; exit 1; }
  tail -2 gpurun_out/clock_sweep.log
  timeout -k 10 240 python3 tools/clock_trace.py gpurun_out/clock_stoi.json -- python3 tools/bench_stoi.py --cells 4096 --reps 40 > gpurun_out/clock_stoi.log 2>&1 || { echo "clock stoi failed"; tail -5 gpurun_out/clock_stoi.log; exit 1; }
  tail -2 gpurun_out/clock_stoi.log
fi
echo call3 done
