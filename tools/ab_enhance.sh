#!/bin/bash
# A/B kernel time of enhance-launch variants (timing-only builds allowed):
# alternate the libraries given as arguments ROUNDS times, each a fresh
# process of tools/time_enhance.py (PAIRS pairs, NFFT).  Prints one JSON line
# per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$@"; do
    CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 ${LIMIT:-240} \
      python tools/time_enhance.py --pairs ${PAIRS:-13} --nfft ${NFFT:-512} --reps ${REPS:-5} || exit 1
  done
done
