#!/bin/bash
# GPU: the whole -m gpu suite, then extra timing tools given as arguments (python scripts)
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=8 > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit $rc; }
for t in "$@"; do
  timeout -k 10 400 python -u $t > $OUT/$(basename $t .py).txt 2>&1 || { tail -5 $OUT/$(basename $t .py).txt; exit 1; }
  grep -v amdgpu.ids $OUT/$(basename $t .py).txt
done
