#!/bin/bash
# A/B timing of kernel builds: scripts/ab.sh SETS lib1 lib2 ...  (SETS e.g. "ADDRESS;DOB,ADDRESS,NAME")
SETS=$1; shift
for lib in "$@"; do
  IFS=';' read -ra S <<< "$SETS"
  for props in "${S[@]}"; do
    echo "== $lib $props"
    DUKEHIP_LIB=$lib PROPS=$props timeout -k 10 120 python3 scripts/ablate_props.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
