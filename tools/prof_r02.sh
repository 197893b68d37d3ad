#!/bin/bash
# One profiling call on the GPU box: kernel stats of the C2 bench leg, then one PMC pass per
# counter group (FETCH_SIZE / WRITE_SIZE for roofline.traffic, SQ issue counters). Only the
# summaries and the k_stream counter rows are kept (gpurun copies back <= 64 MiB). Usage:
#   bash tools/prof_r02.sh <tag> [sq]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=gpurun_out/$1
mkdir -p $T
B="--no-cpu-baseline --no-steal --no-c3 --no-c5 --no-service --steps 1 --warmup 0"
keep() {  # keep the k_stream rows of a pass's counter csv
  f=$(find $T/raw_$1 -name '*counter_collection.csv' | head -n 1)
  mkdir -p $T/pmc_$1
  python3 -c "
import csv,sys
r=csv.DictReader(open('$f')); w=csv.DictWriter(open('$T/pmc_$1/k_stream_counter_collection.csv','w'),r.fieldnames); w.writeheader()
[w.writerow(x) for x in r if 'k_stream' in x.get('Kernel_Name','')]"
  rm -rf $T/raw_$1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/raw_stats -o run -- python3 bench.py $B > $T/bench.json 2> $T/stats.err
cp $(find $T/raw_stats -name '*kernel_stats.csv' | head -n 1) $T/kernel_stats.csv && rm -rf $T/raw_stats
timeout -s KILL 200 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $T/raw_FETCH_SIZE -- python3 bench.py $B > /dev/null 2> $T/f.err
keep FETCH_SIZE
timeout -s KILL 200 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $T/raw_WRITE_SIZE -- python3 bench.py $B > /dev/null 2> $T/w.err
keep WRITE_SIZE
if [ "$2" = sq ]; then
timeout -s KILL 200 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $T/raw_SQ -- python3 bench.py $B > /dev/null 2> $T/sq.err
keep SQ
fi
