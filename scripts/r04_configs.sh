#!/bin/bash
# Round-4 measurement of BASELINE configs[2] at its stated 10M x 10M: the
# bench line (CPU baseline on a bounded sample), kernel trace + stats, one FETCH_SIZE pass,
# a self-launched --gpus 2 gloo rehearsal (two ranks sharing the one GPU: rank_pairs), and
# short default-size lines of the other workloads for frac_bound.
# usage: scripts/r04_configs.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp
mkdir -p $OUT
L="--workload linkage --records 10000000 --no-warm-batch --pcie-steps 0"
timeout -k 10 600 python3 -u bench.py $L --steps 3 --warmup 1 --cpu-seconds 10 \
  > $OUT/bench_linkage_10Mx10M.json 2> $OUT/bench_linkage_10Mx10M.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 bench.py $L --steps 2 --warmup 0 --cpu-seconds 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err
timeout -k 10 600 rocprofv3 --kernel-include-regex "k_score" --pmc FETCH_SIZE --output-format csv \
  -d $OUT/pmc_fetch -o pmc -- python3 bench.py $L --steps 1 --warmup 0 --cpu-seconds 0 \
  > $OUT/pmc_fetch.log 2>&1
DUKEHIP_DIST_BACKEND=gloo timeout -k 10 900 python3 -u bench.py $L --gpus 2 --gather none --steps 2 \
  --warmup 1 --cpu-seconds 0 > $OUT/bench_linkage_10Mx10M_n2_gloo.json 2> $OUT/bench_linkage_10Mx10M_n2_gloo.err
for w in dedup allpairs longtext reference; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 3 --cpu-seconds 0 --pcie-steps 0 \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err
done
echo done
