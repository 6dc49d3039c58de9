#!/bin/bash
# A/B STOI kernel variants on the GPU box with tools/bench_stoi.py (4,096 10-s cells):
#   bash tools/ab_stoi.sh libcse_a.so libcse_b.so ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in "$@"; do
  echo "== $lib"
  CSE_BENCH_NOCHECK=1 CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 python tools/bench_stoi.py --reps ${REPS:-5} 2>/dev/null || exit 1
done
