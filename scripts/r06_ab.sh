#!/bin/bash
# Round-6 A/B of the dedup headline: per named run "name:VAR=value,..." one short bench line
# (env for that run; DUKEHIP_LIB=... picks a library variant from csrc/Makefile).
# usage: scripts/r06_ab.sh OUT workload [run ...]
set -e
OUT=$1; WL=${2:-dedup}
shift 2 || true
export TMPDIR=/tmp
mkdir -p $OUT
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
fi
B="--workload $WL --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0 --no-json-batch ${EXTRA:-}"
for run in "$@"; do
  name=${run%%:*}
  envs=${run#*:}
  (
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [ -n "$e" ] && export "$e"; done
    timeout -k 10 400 python3 -u bench.py $B > $OUT/${WL}_$name.json 2> $OUT/${WL}_$name.err
  )
done
echo done
