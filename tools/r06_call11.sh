#!/bin/bash
# r06 STOI at other input rates: the STOI tests first (incl. the new rates),
# the STOI kernel time on 4,096 10-s cells, then the whole -m gpu suite, smoke
# and the bench line (tools/gpu_check.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stoi.py -m gpu -x -v -s --timeout 300 \
    --timeout-method thread > gpurun_out/stoi_rates_tests.log 2>&1
rc=$?; echo "stoi tests rc=$rc"; tail -16 gpurun_out/stoi_rates_tests.log
[ $rc -eq 0 ] || exit $rc
CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 5 > gpurun_out/stoi_time.log 2>&1 \
    || { echo "bench_stoi failed"; tail -5 gpurun_out/stoi_time.log; exit 1; }
tail -3 gpurun_out/stoi_time.log
bash tools/gpu_check.sh
