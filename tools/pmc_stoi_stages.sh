#!/bin/bash
# LDS instruction and bank-conflict counts of stoi_cells_kernel per ablation
# variant (tools/stoi_ablate.py), one rocprofv3 --pmc pass each:
#   bash tools/pmc_stoi_stages.sh libcse.so libcse_ab1.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_stoi
for lib in "$@"; do
  d=gpurun_out/pmc_stoi/${lib%.so}
  CSE_BENCH_NOCHECK=1 CSE_LIB=classical_speech_enhancement_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $d -o run -- python3 tools/bench_stoi.py --reps 1 > $d.log 2>&1 || { echo "$lib failed"; tail -3 $d.log; exit 1; }
  python3 - "$d" "$lib" <<'PY'
import csv, glob, sys
acc = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "stoi_cells_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
lds, conf = acc.get("SQ_INSTS_LDS", 0), acc.get("SQ_LDS_BANK_CONFLICT", 0)
print(f"{sys.argv[2]}: LDS insts {lds:.4g}  conflict cycles {conf:.4g}  per inst {conf / max(lds, 1):.3f}  VALU {acc.get('SQ_INSTS_VALU', 0):.4g}")
PY
done
