#!/bin/bash
# One A/B GPU call: enhance kernel variants (tools/ab_libs.sh, $NFFT) and STOI
# variants (tools/ab_stoi.sh), each library listed twice in alternation.
#   ENH="libA.so libB.so" STOI="libA.so libC.so" NFFT=1024 bash tools/ab_round.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$ENH" ]; then
  echo "== enhance n_fft ${NFFT:-512}"
  NFFT=${NFFT:-512} bash tools/ab_libs.sh $ENH $ENH || exit 1
fi
if [ -n "$STOI" ]; then
  echo "== stoi"
  bash tools/ab_stoi.sh $STOI $STOI || exit 1
fi
