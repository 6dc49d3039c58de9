#!/bin/bash
# i8 resampler with digit pairs i + j <= 4 (libcse_s4.so) against <= 5 (libcse.so) and the fp64 FIR
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P=classical_speech_enhancement_amd
CSE_LIB=$P/libcse_s4.so CSE_STOI_MF=1 CSE_STOI_DUMP=gpurun_out/stoi_s4.npy CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 3 2>/dev/null || exit 1
CSE_STOI_DUMP=gpurun_out/stoi_f64.npy CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 3 2>/dev/null || exit 1
python -c "import numpy as np; a=np.load('gpurun_out/stoi_s4.npy'); b=np.load('gpurun_out/stoi_f64.npy'); print('max |s4 - fp64|:', float(np.abs(a-b).max()))"
for r in 1 2; do
  echo "== fp64"; CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 5 2>/dev/null || exit 1
  echo "== mf s5"; CSE_STOI_MF=1 CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 5 2>/dev/null || exit 1
  echo "== mf s4"; CSE_LIB=$P/libcse_s4.so CSE_STOI_MF=1 CSE_BENCH_NOCHECK=1 timeout -k 10 300 python tools/bench_stoi.py --reps 5 2>/dev/null || exit 1
done
