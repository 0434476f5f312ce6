#!/bin/bash
# One PMC pass of k_score over a single bench step: scripts/pmc_quick.sh OUTDIR COUNTERS...
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-include-regex "k_score" --pmc "$@" --output-format csv \
  -d $OUT -o pmc -- python3 ${PMC_SCRIPT:-bench.py} ${PMC_ARGS:---steps 1 --warmup 0 --cpu-seconds 0} > $OUT/run.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); d = set()
for r in csv.DictReader(open(f)):
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); d.add(r["Dispatch_Id"])
print("dispatches", len(d))
for k, v in sorted(agg.items()): print(k, v / len(d))
PY
