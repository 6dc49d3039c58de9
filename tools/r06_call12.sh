#!/bin/bash
# r06 generic STFT shapes: the new generic-shape tests (and the mixed-plan
# test) first, then the whole -m gpu suite, smoke and the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 \
    --timeout-method thread -k "generic or one_plan" > gpurun_out/generic_tests.log 2>&1
rc=$?; echo "generic tests rc=$rc"; tail -12 gpurun_out/generic_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh
