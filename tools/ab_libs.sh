#!/bin/bash
# A/B the occupancy variants of libcse on the GPU box (same process shape each).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  CSE_BENCH_NOCHECK=${NOCHECK:-} CSE_LIB=classical_speech_enhancement_amd/$lib timeout -k 10 300 python bench.py --pairs ${PAIRS:-13} --steps ${STEPS:-3} --warmup 1 --nfft ${NFFT:-512} --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('value %.4g evals/s  kernel %.2f ms  step %.2f ms' % (d['value'], d['roofline']['kernel_ms'], d['ms_per_step']))" || exit 1
done
