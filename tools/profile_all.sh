#!/bin/bash
# Kernel trace + PMC passes of the three hot kernels on the GPU box, each pass
# its own rocprofv3 run (gpurun refuses --pmc mixed with trace domains):
#   enhance_kernel<512>  : bench.py (BASELINE config 4 job, 100 pairs) -- the bench line
#   enhance_kernel<1024> : bench.py --nfft 1024
#   stoi_cells_kernel, xcorr_*: tools/bench_sweep.py (full grid, 4 pairs)
#     bash tools/profile_all.sh TAG [what...]     what in {kt512, kt1024, ktsweep, pmc512, pmc1024, pmcstoi, pmcpk, pmcpk1024, pmclds, pmclds1024, pmc512s}
# (pmc512s needs the scalar build: python -c "import __graft_entry__ as g;
#  g.build(out='classical_speech_enhancement_amd/libcse_scalar.so', defines=['CSE_PK=0'])")
# Output under gpurun_out/prof_TAG/; tools/pmc_summary.py turns it into profiles/*.json.
set -o pipefail
TAG=${1:-dev}
shift
WHAT=${*:-kt512 kt1024 ktsweep pmc512 pmc1024 pmcstoi pmcpk pmcpk1024}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B512="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep"
P512="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep"
B1024="bench.py --nfft 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep"
P1024="bench.py --nfft 1024 --steps 1 --warmup 0 --no-cpu-baseline --no-parity --full-grid-steps 0 --no-sweep"
SWEEP="tools/bench_sweep.py --pairs 4 --reps 1"
SQ1="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
# r05: LDS-array busy cycles and LDS-issue stalls (MI355X_MICROARCH.md: SQ_LDS_IDX_ACTIVE =
# all LDS-array cycles, SQ_WAIT_INST_LDS = the LDS-issue share of SQ_WAIT_INST_ANY)
SQLDS="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQF64="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
# r04: how the counters see packed f32 (v_pk_*) instructions
SQPK="SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
# the scalar build of the same sources (CSE_PK=0, every f32 operation its own
# instruction): its F32 class counts minus the product's are the product's
# packed instructions per class (tools/pmc_summary.py packed_counts)
SCALAR_LIB=${SCALAR_LIB:-classical_speech_enhancement_amd/libcse_scalar.so}

kt() {  # name, command...
  local name=$1; shift
  echo "== kernel trace $name"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run -- python3 "$@" > $OUT/kt_$name.log 2>&1 || { echo "kt $name failed"; tail -5 $OUT/kt_$name.log; exit 1; }
  tail -1 $OUT/kt_$name.log
}
pmc() {  # name, counters, command...
  local name=$1 counters=$2; shift 2
  echo "== pmc $name: $counters"
  timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d $OUT/pmc_$name -o run -- python3 "$@" > $OUT/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $OUT/pmc_$name.log; exit 1; }
}
for w in $WHAT; do
  case $w in
    kt512) kt 512 $B512 ;;
    kt1024) kt 1024 $B1024 ;;
    ktsweep) kt sweep $SWEEP ;;
    pmc512) pmc 512_fetch FETCH_SIZE $P512 && pmc 512_write WRITE_SIZE $P512 &&
            pmc 512_sq1 "$SQ1" $P512 && pmc 512_sq2 "$SQ2" $P512 && pmc 512_f64 "$SQF64" $P512 ;;
    pmc1024) pmc 1024_fetch FETCH_SIZE $P1024 && pmc 1024_write WRITE_SIZE $P1024 &&
             pmc 1024_sq1 "$SQ1" $P1024 && pmc 1024_sq2 "$SQ2" $P1024 && pmc 1024_f64 "$SQF64" $P1024 ;;
    pmcstoi) pmc stoi_f64 "$SQF64" $SWEEP && pmc stoi_sq2 "$SQ2" $SWEEP ;;
    pmcpk) pmc pk512 "$SQPK" $P512 ;;
    pmclds) pmc 512_lds "$SQLDS" $P512 ;;
    pmclds1024) pmc 1024_lds "$SQLDS" $P1024 ;;
    pmcpk1024) pmc pk1024 "$SQPK" $P1024 ;;
    pmc512s) CSE_LIB=$SCALAR_LIB pmc s512_pk "$SQPK" $P512 ;;
    *) echo "unknown $w"; exit 1 ;;
  esac
done
echo done
