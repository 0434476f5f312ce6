#!/bin/bash
# Round-5 quick GPU check: the configs[2] parity cases (or the whole GPU suite with FULL=1) and
# an A/B of the linkage bench over named runs "name:VAR=value,VAR=value" (env for that run;
# DUKEHIP_LIB=... picks a library variant from csrc/Makefile).
# usage: scripts/r05_quick.sh OUT records [run ...]
#   e.g. scripts/r05_quick.sh gpurun_out/r05/q7 1000000 default: nodefer:DK_GQ_DEFER=-1
set -e
OUT=$1
REC=${2:-1000000}
shift 2 || true
export TMPDIR=/tmp
mkdir -p $OUT
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
elif [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "config2" -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
fi
B="--workload linkage --records $REC --steps 10 --warmup 2 --cpu-seconds 0 --cpu-single-seconds 0 --no-warm-batch --pcie-steps 0"
for run in "$@"; do
  name=${run%%:*}
  envs=${run#*:}
  (
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [ -n "$e" ] && export "$e"; done
    timeout -k 10 400 python3 -u bench.py $B > $OUT/linkage_$name.json 2> $OUT/linkage_$name.err
  )
done
echo done
