#!/bin/bash
# r04: alignment kernel with the next block's samples prefetched (3 workgroups
# per CU with spills, or 2 without) against the product: kernel traces of a
# 20-pair sweep per library, twice, then the lag parity tests of the winner
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for lib in libcse.so libcse_xpf3.so libcse_xpf2.so; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_xpf_${lib}_$r -o run -- python3 tools/bench_sweep.py --pairs 20 --reps 1 > gpurun_out/kt_xpf_${lib}_$r.log 2>&1 || { echo "kt $lib failed"; tail -3 gpurun_out/kt_xpf_${lib}_$r.log; exit 1; }
  python3 - <<PY
import csv
for row in csv.DictReader(open("gpurun_out/kt_xpf_${lib}_$r/run_kernel_stats.csv")):
    if "xcorr_lag" in row["Name"]:
        print("$lib", "xcorr_lag avg us", round(float(row["AverageNs"])/1e3, 1), "calls", row["Calls"], "total ms", round(float(row["TotalDurationNs"])/1e6, 2))
PY
done
done
for lib in libcse_xpf3.so libcse_xpf2.so; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "align or lag or snr_table" --timeout 300 --timeout-method thread > gpurun_out/parity_$lib.log 2>&1
  echo "parity $lib rc=$?"; tail -1 gpurun_out/parity_$lib.log
done
echo done
