#!/bin/bash
# diagnostics: lifecycle / phase traces and probes of the C2 replay (variant builds in tools/_var)
OUT=gpurun_out/$1; mkdir -p $OUT
DGP_LIB=tools/_var/lib_trace.so timeout -k 10 200 python -u tools/trace_analyze.py 400000 20000 > $OUT/trace1.txt 2>&1 || exit 1
DGP_LIB=tools/_var/lib_trace2.so timeout -k 10 200 python -u tools/trace_phases.py 400000 20000 > $OUT/trace2.txt 2>&1 || exit 1
DGP_LIB=tools/_var/lib_probes.so timeout -k 10 200 python -u tools/stream_prof.py > $OUT/probes_c2.txt 2>&1 || exit 1
DGP_LIB=tools/_var/lib_probes.so timeout -k 10 200 python -u tools/stream_prof.py c3 > $OUT/probes_c3.txt 2>&1 || exit 1
