#!/bin/bash
# r06 short-hop call: the new short-hop parity tests first, then the product
# build's kernel traces + PMC passes again (its sources changed, its ISA did
# not: the committed PMC digest must match this build), then the whole -m gpu
# suite, smoke and the bench line (tools/gpu_check.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 \
    --timeout-method thread -k "short_hop" > gpurun_out/short_hop_tests.log 2>&1
rc=$?; echo "short-hop tests rc=$rc"; tail -8 gpurun_out/short_hop_tests.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r06d} bash tools/r06_call3.sh || exit $?
bash tools/gpu_check.sh
