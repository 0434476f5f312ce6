#!/bin/bash
# PMC passes for k_score on the bench workload (one step).  Each pass is a separate
# rocprofv3 run with --kernel-trace/--stats only besides --pmc (counters in their own run).
# usage: scripts/pmc_profile.sh OUTDIR [bench args...]   (KREGEX: the kernels counted, default
# k_score; configs[4] adds its long-value DP pre-pass, k_long_pre)
set -e
OUT=$1; shift
ARGS=${@:---steps 1 --warmup 0 --cpu-seconds 0 --no-warm-batch --pcie-steps 0}
export TMPDIR=/tmp
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex "${KREGEX:-k_score}" --pmc "$@" --output-format csv \
    -d $OUT/$name -o pmc -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run stall SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32
run l2 TCC_HIT_sum TCC_MISS_sum
