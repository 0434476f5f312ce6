#!/bin/bash
# Round-5 closing measurements at HEAD: the GPU suite, smoke(), and every workload's bench
# line with its CPU baseline.  usage: scripts/r05_final.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
run() {  # name bench-args...
  local name=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
}
run dedup --workload dedup --steps 20 --warmup 5
run dedup_utf16 --workload dedup --utf16-frac 0.01 --steps 10
run linkage --workload linkage --steps 20 --warmup 5
run allpairs_lev --workload allpairs --comparator lev --steps 3
run allpairs_jw --workload allpairs --comparator jw --steps 3
run longtext --workload longtext --steps 5
run reference --workload reference --steps 20
echo done
