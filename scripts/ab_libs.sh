#!/bin/bash
# Same-box A/B of libdukehip builds on the headline bench: scripts/ab_libs.sh ROUNDS LIB_A LIB_B ...
# (a lib path "main" = sesam-duke-microservice_amd/build/libdukehip.so).  Extra bench args in BENCH_ARGS.
R=$1; shift
for r in $(seq 1 $R); do
  for lib in "$@"; do
    path=$lib; [ "$lib" = main ] && path=sesam-duke-microservice_amd/build/libdukehip.so
    DUKEHIP_LIB=$path timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-warm-batch \
      --pcie-steps 0 $BENCH_ARGS > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('$lib', '%.4g' % d['value'], round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['phases_ms_per_step'].items() if k in ('ms_score','ms_emit','ms_gather')})"
  done
done
