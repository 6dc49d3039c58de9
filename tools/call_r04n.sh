#!/bin/bash
# r04: n_fft 1024 radix-2 rotors from a two-row LDS table (no per-element
# select): parity, then a 13-pair A/B against the HEAD build, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/parity_r04n.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/parity_r04n.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  NFFT=1024 STEPS=5 bash tools/ab_libs.sh libcse_base.so libcse.so || exit 1
done
echo done
