#!/bin/bash
# r04 call 2: packed enhance variants at both n_fft + parity + the alignment
# kernel's trace and LDS-conflict PMC (libcse.so = the r03-end sources for the
# alignment kernel, libcse_pkB.so the px32 layout).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh libcse.so libcse_pkA.so libcse_pkB.so libcse.so libcse_pkA.so libcse_pkB.so || exit 1
NFFT=1024 bash tools/ab_libs.sh libcse.so libcse_pkA.so libcse_pkB.so libcse.so libcse_pkB.so || exit 1
for lib in libcse_pkB.so libcse_pkA.so; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$lib.log 2>&1
  rc=$?; echo "parity $lib rc=$rc"; tail -3 gpurun_out/parity_$lib.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
for lib in libcse.so libcse_pkB.so; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_sweep_$lib -o run -- python3 tools/bench_sweep.py --pairs 4 --reps 1 > gpurun_out/kt_sweep_$lib.log 2>&1 || { echo "kt $lib failed"; tail -5 gpurun_out/kt_sweep_$lib.log; exit 1; }
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex xcorr_lag --output-format csv -d gpurun_out/pmc_xc_$lib -o run -- python3 tools/bench_sweep.py --pairs 4 --reps 1 > gpurun_out/pmc_xc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 gpurun_out/pmc_xc_$lib.log; exit 1; }
done
echo done
