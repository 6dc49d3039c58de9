#!/bin/bash
# r04: STOI batch size (GiB of cell waveforms per batch) in the 100-pair sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for gb in 64 96 48 64 96 48; do
  echo "== wave_gb $gb"
  timeout -k 10 300 python -u tools/bench_sweep.py --pairs 100 --reps 2 --wave-gb $gb 2>/dev/null | tail -1 || exit 1
done
echo done
