#!/bin/bash
# GPU suite + short bench lines of the five workloads (+ configs[2] at 10M x 10M when FULL=1).
# usage: scripts/r04_quick.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
for w in dedup linkage allpairs longtext reference; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 5 --cpu-seconds 0 --pcie-steps 0 \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
done
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u bench.py --workload linkage --records 10000000 --no-warm-batch --pcie-steps 0 \
    --steps 3 --warmup 1 --cpu-seconds 10 > $OUT/bench_linkage_10Mx10M.json 2> $OUT/bench_linkage_10Mx10M.err
fi
echo done
