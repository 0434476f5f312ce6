#!/bin/bash
# Round-6 profile of one workload: rocprofv3 kernel trace + stats of a short bench run, then
# PMC passes (each its own run) over the kernels matching KREGEX.
# usage: scripts/r06_prof.sh OUT bench-args...
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 bench.py "$@" --steps 3 --warmup 1 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch \
  --pcie-steps 0 --no-json-batch > $OUT/trace_bench.json 2> $OUT/trace_bench.err
if [ "${PMC:-1}" = 1 ]; then
  KREGEX=${KREGEX:-k_score} bash scripts/pmc_profile.sh $OUT/pmc "$@" --steps 1 --warmup 0 --cpu-seconds 0 \
    --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0 --no-json-batch
fi
echo done
