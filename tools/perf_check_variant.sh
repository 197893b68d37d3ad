#!/bin/bash
# GPU: parity of the default build and of variant V (test_gpu_parity), then C2 / C3 times of both.
# usage: perf_check_variant.sh OUT V
OUT=gpurun_out/$1; V=$2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_default.log 2>&1 || { tail -20 $OUT/pytest_default.log; exit 1; }
tail -1 $OUT/pytest_default.log
DGP_LIB=tools/_var/lib_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$V.log 2>&1 || { tail -20 $OUT/pytest_$V.log; exit 1; }
tail -1 $OUT/pytest_$V.log
timeout -k 10 200 python -u tools/time_c2c3.py 3 > $OUT/time_default.txt 2>&1 || exit 1; echo "== default"; cat $OUT/time_default.txt
DGP_LIB=tools/_var/lib_$V.so timeout -k 10 200 python -u tools/time_c2c3.py 3 > $OUT/time_$V.txt 2>&1 || exit 1; echo "== $V"; cat $OUT/time_$V.txt
