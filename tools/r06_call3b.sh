#!/bin/bash
# r06: the sweep-resident STOI against the solo STOI.  Kernel trace + PMC of a
# 4-pair sweep (tools/profile_all.sh ktsweep pmcstoi), a PMC pass over the solo
# STOI launch (clock held = SQ_BUSY_CYCLES / 32 / time), and the SCLK level
# sampled over a 20-pair sweep and over 40 solo STOI launches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06b}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
bash tools/profile_all.sh $TAG ktsweep pmcstoi || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_stoisolo -o run -- python3 tools/bench_stoi.py --cells 4096 --reps 3 > $OUT/pmc_stoisolo.log 2>&1 || { echo "pmc stoisolo failed"; tail -5 $OUT/pmc_stoisolo.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_stoisolo -o run -- python3 tools/bench_stoi.py --cells 4096 --reps 3 > $OUT/kt_stoisolo.log 2>&1 || { echo "kt stoisolo failed"; tail -5 $OUT/kt_stoisolo.log; exit 1; }
tail -1 $OUT/kt_stoisolo.log
timeout -k 10 300 python3 tools/clock_trace.py gpurun_out/clock_sweep.json -- python3 tools/bench_sweep.py --pairs 20 --reps 1 > gpurun_out/clock_sweep.log 2>&1 || { echo "clock sweep failed"; tail -5 gpurun_out/clock_sweep.log; exit 1; }
tail -2 gpurun_out/clock_sweep.log
timeout -k 10 300 python3 tools/clock_trace.py gpurun_out/clock_stoi.json -- python3 tools/bench_stoi.py --cells 4096 --reps 40 > gpurun_out/clock_stoi.log 2>&1 || { echo "clock stoi failed"; tail -5 gpurun_out/clock_stoi.log; exit 1; }
tail -2 gpurun_out/clock_stoi.log
echo call3b done
