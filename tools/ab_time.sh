#!/bin/bash
# kernel-only A/B of libcse variants (tools/time_enhance.py: no output checks,
# for timing-only builds); one process per library, alternating as listed
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in "$@"; do
  CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 python tools/time_enhance.py --pairs ${PAIRS:-13} --nfft ${NFFT:-512} --reps ${REPS:-8} 2>/dev/null || { echo "$lib failed"; exit 1; }
done
