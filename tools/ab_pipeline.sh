#!/bin/bash
# A/B of the bench's analysis pipelining depth (--pipeline), alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for p in ${PIPES:-2 3 4 2 3 4}; do
  timeout -k 10 300 python bench.py --pipeline $p --steps ${STEPS:-10} --warmup 3 --nfft ${NFFT:-512} --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('pipeline $p: %.4g evals/s  %.2f ms/step  kernel %.2f ms' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms']))" || exit 1
done
