#!/bin/bash
# Per-property ablation of the headline bench: scripts/abl.sh NAME ... (ALL = every property)
for o in "$@"; do
  a="--only $o"; [ "$o" = ALL ] && a=""
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-warm-batch --pcie-steps 0 $a \
    > gpurun_out/abl_$o.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/abl_$o.json').read().strip().splitlines()[-1])
print('$o', '%.4g' % d['value'], round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['phases_ms_per_step'].items()})"
done
