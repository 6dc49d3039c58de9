cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/t_par.log
for q in 1 2; do timeout -k 10 300 python tools/time_noise.py --reps 5 || exit 1; done > gpurun_out/time_noise_g.txt 2>&1; echo "tn rc=$?"; grep prepare gpurun_out/time_noise_g.txt
