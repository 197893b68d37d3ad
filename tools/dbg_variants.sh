#!/bin/bash
# c5mini replay (concurrent mode) under each library variant given
for v in "$@"; do
  echo "== $v"; DGP_LIB=distributed_amd/_var/lib_$v.so timeout -k 10 120 python -u tools/dbg_c5mini.py 2>&1 | tail -1
done
