#!/bin/bash
# r06 second GPU call: VALU instruction-mix micro, the GPU suite on the M2C
# build (libcse.so: bin M/2 evaluated by one wave per frame at both n_fft),
# and 13-pair A/Bs of the enhance launches against the pre-M2C build
# (libcse_base.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 ./tools/micro/valu_mix > gpurun_out/valu_mix.txt 2>&1 || { echo "valu_mix failed"; tail -5 gpurun_out/valu_mix.txt; exit 1; }
cat gpurun_out/valu_mix.txt
NO_BENCH=1 bash tools/gpu_check.sh || exit $?
NFFT=512 ROUNDS=3 bash tools/ab_enhance.sh libcse_base.so libcse.so > gpurun_out/ab_m2c_512.txt 2>&1 || { echo "ab 512 failed"; tail -5 gpurun_out/ab_m2c_512.txt; exit 1; }
cat gpurun_out/ab_m2c_512.txt | grep kernel_ms
NFFT=1024 ROUNDS=3 bash tools/ab_enhance.sh libcse_base.so libcse.so > gpurun_out/ab_m2c_1024.txt 2>&1 || { echo "ab 1024 failed"; tail -5 gpurun_out/ab_m2c_1024.txt; exit 1; }
cat gpurun_out/ab_m2c_1024.txt | grep kernel_ms
