#!/bin/bash
# One GPU session: parity tests, a bench line, a rocprof kernel-trace summary.
# usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/prof.log 2>&1
rc=$?; tail -3 $OUT/prof.log; find $OUT/prof -name '*stats*' | head; exit $rc
