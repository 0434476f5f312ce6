#!/bin/bash
# Round-4 profile of one workload at HEAD: rocprofv3 kernel trace + stats, the PMC passes
# (scripts/pmc_profile.sh), and the bench line with its CPU baseline.
# usage: scripts/r04_profile.sh OUT WHAT [bench args...]   WHAT = trace | pmc | bench | all
set -e
OUT=$1; WHAT=$2; shift 2
ARGS="$@"
export TMPDIR=/tmp
mkdir -p $OUT
if [ $WHAT = trace ] || [ $WHAT = all ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 bench.py $ARGS --steps 3 --warmup 1 --cpu-seconds 0 --no-warm-batch --pcie-steps 0 \
    > $OUT/trace_bench.json 2> $OUT/trace_bench.err
fi
if [ $WHAT = pmc ] || [ $WHAT = all ]; then
  bash scripts/pmc_profile.sh $OUT/pmc $ARGS --steps 1 --warmup 0 --cpu-seconds 0 --no-warm-batch --pcie-steps 0
fi
if [ $WHAT = bench ] || [ $WHAT = all ]; then
  timeout -k 10 600 python3 -u bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
fi
echo done
