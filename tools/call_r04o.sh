#!/bin/bash
# r04: wave_sync as a sched_barrier that lets VALU/SALU/VMEM cross (LDS order
# kept) instead of a full wave_barrier: parity of the variant, then 13-pair
# A/B at both n_fft against the product build, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CSE_LIB=classical_speech_enhancement_amd/libcse_ws.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/parity_r04o.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/parity_r04o.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  STEPS=5 bash tools/ab_libs.sh libcse.so libcse_ws.so || exit 1
  NFFT=1024 STEPS=5 bash tools/ab_libs.sh libcse.so libcse_ws.so || exit 1
done
echo done
