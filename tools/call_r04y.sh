#!/bin/bash
# xcorr FFT image (linear + one swizzled pass instead of the padded images):
# alignment parity with the new libcse.so, then kernel traces of the 4-pair
# sweep for the HEAD build (libcse_xold.so) and the new one, two alternating
# rounds, then one LDS-conflict PMC pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CSE_LIB=classical_speech_enhancement_amd/${TEST_LIB:-libcse.so} timeout -k 10 600 python -u -m pytest \
    ${TESTS:-tests/test_gpu_winners.py tests/test_gpu_stoi.py} -m gpu -x -v -s --timeout 420 \
    --timeout-method thread > gpurun_out/y_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/y_tests.log; exit 1; }
tail -2 gpurun_out/y_tests.log
for r in 1 2; do
  for lib in ${LIBS:-libcse_xold.so libcse.so libcse_xnm.so}; do
    CSE_LIB=classical_speech_enhancement_amd/$lib bash tools/profile_all.sh y_${lib%.so}_$r ktsweep || exit 1
  done
done
for lib in ${LIBS:-libcse_xold.so libcse.so libcse_xnm.so}; do
  CSE_LIB=classical_speech_enhancement_amd/$lib bash tools/profile_all.sh y_${lib%.so} pmcstoi || exit 1
done
echo done
