#!/bin/bash
# r05 occupancy evidence: kernel trace (VGPRs, LDS, ms)
# and one SQ pass (waves, wave cycles, wait shares) of enhance-launch builds,
# each its own rocprofv3 run, on tools/time_enhance.py (13 pairs, n_fft 512).
#   b3 : r04 kernel, OMLSA hop 128 only (timing build)
#   p3 : b3 + tools/probes/occupancy_probe4.patch's LDS cuts (<= 40 KB), 3 waves/SIMD
#   p4 : p3 at 4 waves/SIMD (128 VGPRs, no spill)
#   s3 / s4 : the full kernel with CSE_SPLIT_T=1 at 3 / 4 waves/SIMD
#     bash tools/occupancy_probe.sh lib...      (names under the package dir)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/occ
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for lib in "$@"; do
  n=${lib%.so}; n=${n#libcse_}
  export CSE_LIB=classical_speech_enhancement_amd/$lib
  echo "== $lib"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$n -o run -- \
      python3 tools/time_enhance.py --reps 3 > $OUT/kt_$n.log 2>&1 || { echo "kt $n failed"; tail -5 $OUT/kt_$n.log; exit 1; }
  tail -1 $OUT/kt_$n.log
  timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc_$n -o run -- \
      python3 tools/time_enhance.py --reps 1 > $OUT/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $OUT/pmc_$n.log; exit 1; }
done
echo done
