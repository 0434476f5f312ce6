#!/bin/bash
# Round-6 profiles at HEAD: per workload a rocprofv3 kernel trace + stats of a short bench
# run and the PMC passes (scripts/pmc_profile.sh); scripts/summarize_profiles.py turns them
# into profiles/pmc_<key>.json afterwards (on the host: only gpurun_out/ comes back).
# usage: scripts/r06_head.sh OUT name:bench-args... (args comma-separated)
#   e.g. scripts/r06_head.sh gpurun_out/r06/head dedup:--workload,dedup linkage:--workload,linkage
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
(while sleep 50; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
for spec in "$@"; do
  name=${spec%%:*}
  args=$(echo "${spec#*:}" | tr ',' ' ')
  mkdir -p $OUT/$name
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name/trace -o trace -- \
    python3 bench.py $args --steps 3 --warmup 1 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0 \
    --no-json-batch > $OUT/$name/trace_bench.json 2> $OUT/$name/trace_bench.err
  KREGEX="k_score" bash scripts/pmc_profile.sh $OUT/$name/pmc $args --steps 1 --warmup 0 --cpu-seconds 0 --cpu-single-seconds 0 \
    --no-warm-batch --pcie-steps 0 --no-json-batch --phase-steps 0
  rm -f $OUT/$name/trace/*kernel_trace.csv  # the stats and counters are what is kept (gpurun_out <= 64 MiB)
  du -sh $OUT/$name
  echo "$name done"
done
echo done
