#!/bin/bash
# GPU: stream-engine parity (test_gpu_parity + service) then C2 / C3 wall times.
# usage: tools/gpu_quick.sh OUTDIR [pytest files...]
OUT=$1; shift
mkdir -p $OUT
T=${@:-tests/test_gpu_parity.py}
timeout -k 10 500 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python -u tools/time_c2c3.py 2 > $OUT/time.txt 2>&1; rc=$?; cat $OUT/time.txt | grep -v amdgpu.ids; exit $rc
