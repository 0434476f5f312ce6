#!/bin/bash
# PMC A/B of the configs[2] scoring kernels at 1M x 1M: one SQ pass per library variant.
# usage: scripts/r05_pmc_ab.sh OUT name=lib ...   (lib "" = the default build; DK_GQ=0 via name "old")
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
for nv in "$@"; do
  n=${nv%%=*}; lib=${nv#*=}
  env=""
  [ "$n" = old ] && export DK_GQ=0 || unset DK_GQ
  if [ -n "$lib" ]; then export DUKEHIP_LIB=$lib; else unset DUKEHIP_LIB; fi
  PMC_ARGS="--workload linkage --steps 1 --warmup 0 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0" \
    timeout -k 10 200 bash scripts/pmc_quick.sh $OUT/$n $C > $OUT/$n.txt
done
echo done
