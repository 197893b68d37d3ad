#!/bin/bash
# GPU: C2 / C3 wall times of the default build under DGP_STREAM_DEBUG values (executor
# counts in bits 8..11), then of variant libraries. usage: perf_knobs.sh OUT "dbg1 dbg2" var1 var2 ...
OUT=gpurun_out/$1; DBGS=$2; shift 2; mkdir -p $OUT
for d in $DBGS; do
  DGP_STREAM_DEBUG=$d timeout -k 10 200 python -u tools/time_c2c3.py 2 > $OUT/time_dbg$d.txt 2>&1 || exit 1
  echo "== dbg $d"; cat $OUT/time_dbg$d.txt
done
for v in "$@"; do
  DGP_LIB=tools/_var/lib_$v.so timeout -k 10 200 python -u tools/time_c2c3.py 2 > $OUT/time_$v.txt 2>&1 || exit 1
  echo "== $v"; cat $OUT/time_$v.txt
done
