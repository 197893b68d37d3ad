#!/bin/bash
# Time the C2 replay under diagnostic library variants (distributed_amd/_var/lib_<name>.so).
# usage (GPU): tools/knob_sweep.sh OUTDIR name...   ("base" = the in-tree libdgplace.so)
OUT=$1; shift
mkdir -p $OUT
for n in "$@"; do
  if [ "$n" = base ]; then L=""; else L=distributed_amd/_var/lib_$n.so; fi
  DGP_LIB=$L timeout -k 10 120 python -u tools/stream_prof.py > $OUT/$n.txt 2>&1 || { echo "$n failed"; cat $OUT/$n.txt | tail -5; exit 1; }
  echo "$n: $(grep run_rounds $OUT/$n.txt) | $(grep 'EXE claim' $OUT/$n.txt | awk '{print "exe", $NF}') | $(grep 'REG busy' $OUT/$n.txt | awk '{print "reg", $NF}') | $(grep 'SEQ busy' $OUT/$n.txt | awk '{print "seq", $NF}') | $(grep 'EXE idle' $OUT/$n.txt | awk '{print "idle", $NF}')"
done
