set -o pipefail
O=gpurun_out/r05w; mkdir -p $O; export TMPDIR=/tmp
for cfg in "1000000 1024" "1000000 64" "250000 1024"; do
  set -- $cfg
  for C in WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    t=$(echo $C | cut -c1-12)_$1_$2
    timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $O/$t -o run -- python3 tools/wr_probe.py $1 $2 > $O/$t.log 2>&1 || exit 1
  done
done
