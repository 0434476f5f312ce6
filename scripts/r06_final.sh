#!/bin/bash
# Round-6 closing measurements at HEAD (one capture for the round): the GPU suite, smoke(),
# and each named workload's bench line with its CPU baseline.
# usage: scripts/r06_final.sh OUT [tests] name ...   (names: see run_one below)
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
(while sleep 50; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
run() {  # name bench-args...
  local name=$1; shift
  timeout -k 10 900 python3 -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  echo "$name done"
}
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
      tail -1 $OUT/gputest.log
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
      tail -1 $OUT/smoke.log ;;
    dedup) run dedup --workload dedup --steps 20 --warmup 5 ;;
    dedup_utf16) run dedup_utf16 --workload dedup --utf16-frac 0.01 --steps 10 ;;
    linkage) run linkage --workload linkage --steps 20 --warmup 5 ;;
    linkage_10m) run linkage_10m --workload linkage --records 10000000 --steps 3 --warmup 1 --pcie-steps 0 ;;
    allpairs_lev) run allpairs_lev --workload allpairs --comparator lev --steps 3 ;;
    allpairs_jw) run allpairs_jw --workload allpairs --comparator jw --steps 3 ;;
    longtext) run longtext --workload longtext --steps 5 ;;
    reference) run reference --workload reference --steps 20 ;;
  esac
done
echo done
