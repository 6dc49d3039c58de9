#!/bin/bash
# A/B: the hops' analysis chains on forked streams vs one stream (CSE_SERIAL_HOPS=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARS:-1 0 1 0}; do
  CSE_SERIAL_HOPS=$v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --nfft ${NFFT:-512} --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('serial_hops=$v: %.4g evals/s  %.2f ms/step  kernel %.2f ms' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms']))" || exit 1
done
