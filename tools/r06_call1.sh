#!/bin/bash
# r06 first GPU call: the GPU suite + smoke + bench line (tools/gpu_check.sh),
# then the chip-wide VALU calibration and the alignment head timings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 120 ./tools/micro/valu_cal > gpurun_out/valu_cal.txt 2>&1 || { echo "valu_cal failed"; tail -5 gpurun_out/valu_cal.txt; exit 1; }
cat gpurun_out/valu_cal.txt | grep -v JSON
timeout -k 10 120 python -u tools/time_alignment.py gpurun_out/alignment_heads.json > gpurun_out/alignment_heads.log 2>&1 || { echo "time_alignment failed"; tail -5 gpurun_out/alignment_heads.log; exit 1; }
cat gpurun_out/alignment_heads.log
