#!/bin/bash
# GPU: parity of the default build, then C2 / C3 wall times of the default build and variants
OUT=gpurun_out/$1; shift; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/time_c2c3.py 3 > $OUT/time_default.txt 2>&1 || exit 1; cat $OUT/time_default.txt
for v in "$@"; do
  DGP_LIB=tools/_var/lib_$v.so timeout -k 10 200 python -u tools/time_c2c3.py 3 > $OUT/time_$v.txt 2>&1 || exit 1
  echo "== $v"; cat $OUT/time_$v.txt
done
