#!/bin/bash
# One GPU-box check: the -m gpu suite (or the tests named in $TESTS), smoke,
# then the bench line.  Each GPU step has its own time limit; a step that ends
# in a fault, abort, segfault or time limit stops the script (exit codes 124,
# 134, 137, 139 and signals), an ordinary test failure (rc 1) does not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5}
stop() { case $1 in 0|1) return 1 ;; *) return 0 ;; esac; }
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 420 \
    --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
if stop $rc; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/smoke.log
if stop $rc2; then exit $rc2; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_LIMIT:-420} python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc3=$?; echo "bench rc=$rc3"; tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $(( rc | rc2 | rc3 ))
