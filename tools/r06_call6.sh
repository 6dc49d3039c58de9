#!/bin/bash
# r06: which SQ_INSTS_VALU_* classes gfx950's rocprofv3 offers, then one pass
# of the integer / conversion classes over the 512 enhance launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r06c
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/list_avail.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1
grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_INSTS_SALU[A-Z0-9_]*\|SQ_INST_LEVEL[A-Z0-9_]*" $OUT/list_avail.txt | sort -u | tee $OUT/valu_counters.txt
C=$(grep -E "^SQ_INSTS_VALU_(INT32|INT64|CVT|TRANS_F32|ADD_F32|MUL_F32|FMA_F32)$" $OUT/valu_counters.txt | head -4 | tr '\n' ' ')
echo "pass: $C"
P512="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep"
if [ -n "$C" ]; then
  timeout -s KILL 240 rocprofv3 --pmc $C SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_512_int -o run -- python3 $P512 > $OUT/pmc_512_int.log 2>&1 || { echo "pmc int failed"; tail -5 $OUT/pmc_512_int.log; exit 1; }
fi
echo call6 done
