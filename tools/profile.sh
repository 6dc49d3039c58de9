#!/bin/bash
# Profile bench.py on the GPU box: kernel trace/stats + PMC passes (each its own run).
#   bash tools/profile.sh TAG [PAIRS]
set -o pipefail
TAG=${1:-dev}
PAIRS=${2:-4}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --steps 2 --warmup 1 --pairs $PAIRS --no-cpu-baseline"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $B > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log
shift 2
for pass in "$@"; do
  echo "== pmc $pass"
  timeout -k 10 300 rocprofv3 --pmc ${pass//,/ } --output-format csv -d $OUT/pmc_${pass%%,*} -o run -- python3 bench.py --steps 1 --warmup 0 --pairs $PAIRS --no-cpu-baseline > $OUT/pmc_${pass%%,*}.log 2>&1 || { echo "pmc $pass failed"; tail -5 $OUT/pmc_${pass%%,*}.log; exit 1; }
done
echo done
