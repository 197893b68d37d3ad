#!/bin/bash
# One GPU session: parity tests, a bench line, a rocprof kernel-trace summary.
# usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=8 > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/prof.log 2>&1
rc=$?; tail -3 $OUT/prof.log; ls $OUT/prof; [ $rc -ne 0 ] && exit $rc
# HBM traffic of the C2 replay: one counter per pass (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu-baseline --no-steal --no-c3 --no-c5 --no-variants --no-service --steps 1 --warmup 0 > $OUT/pmc_$C.log 2>&1
  rc=$?; tail -2 $OUT/pmc_$C.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
