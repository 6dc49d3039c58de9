#!/bin/bash
# r04: host-side profile of the 100-pair sweep (cProfile of the timed STOI sweep)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_sweep.py --pairs 100 --reps 1 --profile > gpurun_out/sweep_prof.json 2> gpurun_out/sweep_prof.txt || { echo "failed"; tail -5 gpurun_out/sweep_prof.txt; exit 1; }
cat gpurun_out/sweep_prof.json
echo done
