#!/bin/bash
# GPU session part 1: the full -m gpu suite and one default bench line; the full-graph C5 CPU
# baseline (tools/c5_cpu_full.py, host cores only) runs beside them.
# usage: tools/gpu_round_a.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/c5_cpu_full.py > $OUT/c5_cpu_full.json 2> $OUT/c5_cpu_full.err &
CPID=$!
echo "== pytest gpu"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=8 > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && { kill $CPID; exit $rc; }
echo "== bench"
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log; [ $rc -ne 0 ] && { kill $CPID; exit $rc; }
echo "== c5 cpu full (waiting)"
wait $CPID; rc=$?; cat $OUT/c5_cpu_full.json; exit $rc
