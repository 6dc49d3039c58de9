#!/bin/bash
# r04: finish and iir without per-access branches, loads a block ahead: noise
# parity, kernel trace of the 512 bench, then a 100-pair A/B of ms/step
# against the HEAD build (libcse_base.so), alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/parity_r04k.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/parity_r04k.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_r04k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep > gpurun_out/kt_r04k.log 2>&1 || { echo "kt failed"; tail -5 gpurun_out/kt_r04k.log; exit 1; }
PAIRS=100 STEPS=5 bash tools/ab_libs.sh libcse_base.so libcse.so libcse_base.so libcse.so || exit 1
echo done
