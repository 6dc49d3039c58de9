cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
(bash tools/ab_stoi.sh libcse_r04.so libcse.so libcse_r04.so libcse.so) > gpurun_out/ab_stoi_r05a.txt 2>&1; echo "ab rc=$?"; grep -o '"ms_per_launch": [0-9.]*' gpurun_out/ab_stoi_r05a.txt
CSE_LIB=classical_speech_enhancement_amd/libcse_stamps.so timeout -k 10 200 python tools/stoi_stages.py > gpurun_out/stoi_stages2.json 2>&1; echo "stages rc=$?"; grep -A1 '"share"\|cycles_per_cell' gpurun_out/stoi_stages2.json | grep -v "^--" | tr -d '\n'; echo
timeout -k 10 400 python -u -m pytest tests/test_gpu_stoi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_stoi.log 2>&1; echo "stoi tests rc=$?"; tail -2 gpurun_out/t_stoi.log
