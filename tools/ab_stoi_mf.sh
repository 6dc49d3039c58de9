#!/bin/bash
# The STOI resampler paths on one box: the i8-sliced MFMA FIR (default for
# clipped cells with CSE_STOI_MF=1) against the fp64 FIR: per-cell scores
# compared, then alternating timings (tools/bench_stoi.py, 4,096 10-s cells)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CSE_STOI_MF=1 CSE_STOI_DUMP=gpurun_out/stoi_mf.npy timeout -k 10 300 python tools/bench_stoi.py --reps 3 || exit 1
CSE_STOI_DUMP=gpurun_out/stoi_f64.npy timeout -k 10 300 python tools/bench_stoi.py --reps 3 || exit 1
python -c "import numpy as np; a=np.load('gpurun_out/stoi_mf.npy'); b=np.load('gpurun_out/stoi_f64.npy'); print('max |mf - fp64| over', len(a), 'cells:', float(np.abs(a-b).max()))"
for r in 1 2; do
  for v in 0 1; do
    echo "== CSE_STOI_MF=$v"
    CSE_STOI_MF=$v timeout -k 10 300 python tools/bench_stoi.py --reps ${REPS:-5} || exit 1
  done
done
CSE_STOI_MF=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_stoi.py -m gpu -x -q --timeout 300 > gpurun_out/stoi_tests_mf.log 2>&1
echo "stoi tests with CSE_STOI_MF=1: rc=$?"; tail -3 gpurun_out/stoi_tests_mf.log
