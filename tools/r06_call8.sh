#!/bin/bash
# r06: OMLSA's L from a stager row of log2(gamma log2 e) at n_fft 512 (one
# transcendental less per bin): 13-pair A/B against HEAD's build, then the
# GPU suite on it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
NFFT=512 ROUNDS=3 bash tools/ab_enhance.sh libcse_base.so libcse.so > gpurun_out/ab_logrow.txt 2>&1 || { echo "ab failed"; tail -5 gpurun_out/ab_logrow.txt; exit 1; }
grep kernel_ms gpurun_out/ab_logrow.txt
NO_BENCH=1 bash tools/gpu_check.sh
