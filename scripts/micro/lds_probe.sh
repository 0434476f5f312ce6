#!/bin/bash
# the LDS probe microbenchmark on the GPU box -- timing run, then one PMC
# pass (its own run) -- and the per-variant summary (scripts/micro/lds_probe_summary.py).
# usage: scripts/micro/lds_probe.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 60 ./scripts/micro/lds_probe > $OUT/timing.jsonl
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
  --output-format csv -d $OUT/pmc -o pmc -- ./scripts/micro/lds_probe > $OUT/pmc_run.log 2>&1
python3 scripts/micro/lds_probe_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
