#!/bin/bash
# r04 call d: OMLSA's speech presence divided by q (one multiply less per bin):
# 13-pair A/B against the previous build, parity, then (if asked) the enhance
# PMC passes and the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh libcse_prev.so libcse.so libcse_prev.so libcse.so libcse_prev.so libcse.so || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r04d.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/parity_r04d.log
[ $rc -eq 0 ] || exit $rc
[ -n "$PROFILE" ] || exit 0
bash tools/profile_all.sh r04d kt512 pmc512 pmcpk pmc512s kt1024 pmc1024 || exit 1
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench.json
exit $rc
