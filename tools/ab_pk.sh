#!/bin/bash
# r04: packed-f32 (CSE_PK) enhance A/B + its parity, then the HEAD check.
#   1. tools/micro/pk_occ (packed vs scalar issue at 1-4 waves/SIMD)
#   2. 13-pair enhance<512> kernel time, libs alternating (tools/ab_libs.sh)
#   3. tests/test_gpu_parity.py against each packed lib
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -x tools/micro/pk_occ ]; then
  timeout -k 10 60 tools/micro/pk_occ > gpurun_out/pk_occ.txt 2>&1 || { echo "pk_occ failed"; cat gpurun_out/pk_occ.txt; exit 1; }
  cat gpurun_out/pk_occ.txt
fi
LIBS=${LIBS:-"libcse_base.so libcse_pk.so libcse_pkd.so"}
bash tools/ab_libs.sh $LIBS $LIBS || exit 1
for lib in ${PARITY_LIBS:-libcse_pkd.so}; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$lib.log 2>&1
  rc=$?; echo "parity $lib rc=$rc"; tail -3 gpurun_out/parity_$lib.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
