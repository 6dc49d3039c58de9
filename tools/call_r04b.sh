#!/bin/bash
# r04: parity of the current libcse.so (alignment kernel with mirror-pair
# ownership), then kernel traces and PMC passes of the enhance<512> kernel
# (product = packed build, plus the scalar build's counts).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r04b.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/parity_r04b.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_all.sh ${TAG:-r04a} ${WHAT:-kt512 ktsweep pmc512 pmcpk pmc512s}
