#!/bin/bash
# r06: the box's clock and power state, then the bench line again (the
# round's earlier boxes ran the enhance launch at 164-165 ms, call 4's at 193).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
{
  echo "== rocm-smi --showclocks"; timeout 20 rocm-smi --showclocks 2>&1 | head -30
  echo "== rocm-smi --showpower --showmaxpower --showtemp"; timeout 20 rocm-smi --showpower --showmaxpower --showtemp 2>&1 | head -30
  echo "== amd-smi metric"; timeout 30 amd-smi metric -c -p -t 2>&1 | head -60
  echo "== pp_dpm_sclk"; cat /sys/class/drm/card*/device/pp_dpm_sclk 2>&1 | head -20
  echo "== gpu_metrics"; ls -la /sys/class/drm/card*/device/gpu_metrics 2>&1 | head
} > gpurun_out/box_state.txt 2>&1
cat gpurun_out/box_state.txt | head -80
timeout -k 10 420 python3 tools/clock_trace.py gpurun_out/clock_bench.json -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo "bench failed"; tail -5 gpurun_out/bench5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench5.json').read().strip().splitlines()[-2 if open('gpurun_out/bench5.json').read().strip().splitlines()[-1].startswith('clock_trace') else -1])
print('ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'full', d['full_grid']['kernel_ms'], 'sweep', d['sweep']['wall_s'])"
tail -1 gpurun_out/bench5.json
