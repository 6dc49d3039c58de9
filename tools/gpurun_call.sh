cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=3 LIMIT=200 bash tools/ab_enhance.sh libcse_r04.so libcse_t0.so libcse.so > gpurun_out/ab_r05e.txt 2>&1; echo "ab rc=$?"; grep kernel_ms gpurun_out/ab_r05e.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_t1.log 2>&1; echo "t1 tests rc=$?"; tail -2 gpurun_out/t_t1.log
