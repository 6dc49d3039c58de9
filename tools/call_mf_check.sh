#!/bin/bash
# The i8 STOI resampler's validation (scores vs the fp64 FIR, timing, STOI
# tests with it on) and the full check of the default build in one call
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/ab_stoi_mf.sh > gpurun_out/ab_stoi_mf.txt 2>&1; rc=$?
cat gpurun_out/ab_stoi_mf.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_check.sh
