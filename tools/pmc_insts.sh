#!/bin/bash
# GPU: instruction / cycle counters of the C2 stream replay (k_stream), one pass per set.
# usage: tools/pmc_insts.sh OUTDIR [n_tasks]
OUT=$1; N=${2:-1000000}
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 tools/stream_once.py $N > $OUT/pmc$i.log 2>&1
  rc=$?; tail -2 $OUT/pmc$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
