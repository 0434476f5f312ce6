#!/bin/bash
# A/B of k_score_grouped builds on configs[2] (1M x 1M): scripts/ab_grouped.sh OUTDIR name...
# (name "main" = the in-tree library; others = build/var/libdukehip_<name>.so)
OUT=$1; shift
mkdir -p $OUT
for n in "$@"; do
  if [ "$n" = main ]; then unset DUKEHIP_LIB; else export DUKEHIP_LIB=$PWD/sesam-duke-microservice_amd/build/var/libdukehip_$n.so; fi
  timeout -k 10 200 python3 -u bench.py --workload linkage --steps 10 --cpu-seconds 0 \
    --no-warm-batch --pcie-steps 0 ${AB_ARGS} > $OUT/$n.json 2> $OUT/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4e' % d['value'], round(d['ms_per_step'],2), round(d['phases_ms_per_step']['ms_score'],2))"
done
