#!/bin/bash
# r04: the CPU baseline leg at 1, 4 and 16 processes (host cores only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cpu_scaling.py --budget 10 > gpurun_out/cpu_scaling.json 2> gpurun_out/cpu_scaling.err || { tail -5 gpurun_out/cpu_scaling.err; exit 1; }
cat gpurun_out/cpu_scaling.json
echo done
