#!/bin/bash
# GPU: parity of the replay engine, then the C2 / C3 stream profiles (one line each).
# usage: tools/perf_check.sh OUTDIR [pytest files...]
OUT=$1; shift
mkdir -p $OUT
T=${@:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for w in c2 c3; do
  if [ $w = c2 ]; then A=""; else A=c3; fi
  timeout -k 10 200 python -u tools/stream_prof.py $A > $OUT/prof_$w.txt 2>&1 || { tail -5 $OUT/prof_$w.txt; exit 1; }
  echo "$w: $(grep run_rounds $OUT/prof_$w.txt) | $(grep 'EXE claim' $OUT/prof_$w.txt | awk '{print "exe", $NF}') | $(grep 'REG busy' $OUT/prof_$w.txt | awk '{print "reg", $NF}') | $(grep 'SEQ busy' $OUT/prof_$w.txt | awk '{print "seq", $NF}') | $(grep 'EXE idle' $OUT/prof_$w.txt | awk '{print "idle", $NF}') | $(grep 'REG window full' $OUT/prof_$w.txt | awk '{print "winfull", $NF}')"
done
