#!/bin/bash
# Round-4 measurement of configs[2] at 1M x 1M: FETCH_SIZE calibration, kernel trace + stats,
# PMC passes, and the bench line with its CPU baseline.  usage: scripts/r04_linkage_profile.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp
R=$PWD
mkdir -p $OUT
( cd /tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
    -d $R/$OUT/fetch_calib -o pmc -- $R/scripts/micro/fetch_calib > $R/$OUT/fetch_calib.log 2>&1 )
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 bench.py --workload linkage --steps 5 --cpu-seconds 0 --no-warm-batch --pcie-steps 0 \
  > $OUT/trace_bench.json 2> $OUT/trace_bench.err
bash scripts/pmc_profile.sh $OUT/pmc --workload linkage --steps 1 --warmup 0 --cpu-seconds 0 --no-warm-batch --pcie-steps 0
timeout -k 10 300 python3 bench.py --workload linkage --steps 10 > $OUT/bench_linkage.json 2> $OUT/bench_linkage.err
echo done
