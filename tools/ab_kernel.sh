#!/bin/bash
# A/B one kernel's average duration across libcse variants on the GPU box:
#   KERNEL=xcorr_lag_kernel bash tools/ab_kernel.sh libcse_a.so libcse_b.so ...
# each lib under rocprofv3 --kernel-trace --stats of tools/bench_sweep.py (full grid, 4 pairs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
K=${KERNEL:-xcorr_lag_kernel}
for lib in "$@"; do
  d=gpurun_out/ab_${lib%.so}
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/bench_sweep.py --pairs ${PAIRS:-4} --reps 1 > $d.log 2>&1 || { echo "$lib failed"; tail -5 $d.log; exit 1; }
  python3 - "$d" "$K" "$lib" <<'PY'
import csv, glob, sys
d, k, lib = sys.argv[1:]
for f in glob.glob(d + "/**/run_kernel_stats.csv", recursive=True) + glob.glob(d + "/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if k in r["Name"]:
            print(lib, r["Name"][:50], "calls", r["Calls"], "avg_ms %.4f" % (float(r["AverageNs"]) / 1e6))
    break
PY
done
