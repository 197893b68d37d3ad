#!/bin/bash
# GPU session part 2: rocprof kernel stats of a short bench, then the HBM traffic of the C2
# replay (one counter per pass: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
# usage: tools/gpu_round_b.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; tail -2 $OUT/prof.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu-baseline --no-steal --no-c3 --no-c5 --no-variants --no-service --steps 1 --warmup 0 > $OUT/pmc_$C.log 2>&1
  rc=$?; tail -1 $OUT/pmc_$C.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
exit 0
