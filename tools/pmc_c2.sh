#!/bin/bash
# GPU: HBM traffic of the C2 replay, one counter per pass (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
# usage: tools/pmc_c2.sh OUTDIR
OUT=$1; mkdir -p $OUT; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu-baseline --no-steal --no-c3 --no-c5 --no-variants --no-service --no-latency --steps 1 --warmup 0 > $OUT/pmc_$C.log 2>&1 || exit 1
done
