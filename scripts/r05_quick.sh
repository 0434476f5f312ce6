#!/bin/bash
# Round-5 quick GPU check: the configs[2] parity cases and an A/B of the linkage bench
# (k_score_gq vs k_score_grouped, and kernel variants from csrc/Makefile gvariant).
# usage: scripts/r05_quick.sh OUT [records] [variant names...]
set -e
OUT=$1
REC=${2:-1000000}
shift 2 || true
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "config2" -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
B="--workload linkage --records $REC --steps 10 --warmup 2 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0"
DK_GQ=0 timeout -k 10 400 python3 -u bench.py $B > $OUT/linkage_old.json 2> $OUT/linkage_old.err
timeout -k 10 400 python3 -u bench.py $B > $OUT/linkage_gq.json 2> $OUT/linkage_gq.err
for v in "$@"; do
  DUKEHIP_LIB=sesam-duke-microservice_amd/build/var/libdukehip_$v.so timeout -k 10 400 python3 -u bench.py $B > $OUT/linkage_$v.json 2> $OUT/linkage_$v.err
done
echo done
