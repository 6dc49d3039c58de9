cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
NO_BENCH=1 bash tools/gpu_check.sh; rc=$?; echo "gpu_check rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
CSE_LIB=classical_speech_enhancement_amd/libcse_s3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_s3.log 2>&1; echo "s3 tests rc=$?"; tail -3 gpurun_out/t_s3.log
bash tools/occupancy_probe.sh libcse.so libcse_b3.so libcse_p3.so libcse_p4.so libcse_s3.so libcse_s4.so
