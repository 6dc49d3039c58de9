#!/bin/bash
# One rocprofv3 --pmc pass per library variant (same bench shape), enhance kernel totals.
#   bash tools/pmc_libs.sh "COUNTERS" lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
C="$1"; shift
for lib in "$@"; do
  d=gpurun_out/pmc_libs/${lib%.so}
  mkdir -p $d
  CSE_BENCH_NOCHECK=1 CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 0 --pairs ${PAIRS:-8} --nfft ${NFFT:-512} --no-cpu-baseline --no-parity > $d.log 2>&1 || { echo "$lib failed"; tail -3 $d.log; exit 1; }
  python - "$d" "$lib" <<'PY'
import csv, glob, sys
acc = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "enhance_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(sys.argv[2], " ".join(f"{k}={v:.3g}" for k, v in sorted(acc.items())))
PY
done
