#!/bin/bash
# A/B of bench.py lines under environment variants, alternated ROUNDS times,
# each a fresh process; prints ms_per_step, the enhance-kernel ms and the
# analysis chain's span per variant.  Optional parity tests first ($TESTS).
#   VARIANTS="CSE_PREP_PRIORITY=-1 CSE_PREP_PRIORITY=0" bash tools/ab_bench.sh
# (a variant is NAME=VALUE[,NAME=VALUE...], or "-" for the plain environment)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 \
      --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
B=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep}
i=0
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:--}; do
    i=$((i + 1))
    out=gpurun_out/ab_bench_$i.json
    if [ "$v" = "-" ]; then
      timeout -k 10 ${LIMIT:-300} python bench.py $B > $out 2> $out.err || { echo "$v failed"; tail -5 $out.err; exit 1; }
    else
      env ${v//,/ } timeout -k 10 ${LIMIT:-300} python bench.py $B > $out 2> $out.err || { echo "$v failed"; tail -5 $out.err; exit 1; }
    fi
    python - "$out" "$v" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["ranks"]["per_rank"][0]
print(f"{sys.argv[2]:32s} ms/step {d['ms_per_step']:.3f}  kernel {r['kernel_ms']:.3f}  "
      f"analysis {r['analysis_ms']:.3f}  value {d['value']:.4g}")
EOF
  done
done
