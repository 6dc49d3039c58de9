#!/bin/bash
# r04 call c: VALU peak micro, STOI parity of the product lib (i8 path removed),
# the 1024 workgroup-size A/B with the launch bounds as waves per SIMD (ADVICE
# r03), the remaining kernel traces / PMC passes, then the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/micro/valu_peak > gpurun_out/valu_peak.txt 2>&1 || { echo "valu_peak failed"; cat gpurun_out/valu_peak.txt; exit 1; }
cat gpurun_out/valu_peak.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_stoi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/stoi_r04c.log 2>&1
rc=$?; echo "stoi tests rc=$rc"; tail -3 gpurun_out/stoi_r04c.log
[ $rc -eq 0 ] || exit $rc
NFFT=1024 bash tools/ab_libs.sh libcse.so libcse_w6.so libcse_w12.so libcse.so libcse_w6.so libcse_w12.so || exit 1
bash tools/profile_all.sh r04a kt1024 pmc1024 pmcstoi || exit 1
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.json
exit $rc
