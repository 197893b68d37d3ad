#!/bin/bash
# Instruction statistics of the stream executor role (entry_exe<true>) in the current sources.
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
  --offload-device-only $@ -o /tmp/dev.co /root/repo/distributed_amd/csrc/dgplace.hip 2>/dev/null
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/dev.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/dev950.o
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 /tmp/dev950.o > /tmp/dev.s
for f in entry_exeILb1EEEvv entry_regILb1EEEvv entry_wlkILb1EEEvv entry_stageILi0EEEvv entry_stageILi1EEEvv; do
  a=$(grep -n "${f}>:" /tmp/dev.s | cut -d: -f1)
  b=$(awk -v s=$a 'NR>s && />:$/ {print NR; exit}' /tmp/dev.s)
  sed -n "${a},${b}p" /tmp/dev.s > /tmp/fn.s
  body=$(grep -n "scratch_" /tmp/fn.s | awk -F: -v n=$(wc -l < /tmp/fn.s) '$1>80 && $1<n-120' | wc -l)
  echo "$f lines $(wc -l < /tmp/fn.s) scratch $(grep -c scratch_ /tmp/fn.s) (body $body) readlane $(grep -c v_readlane /tmp/fn.s) writelane $(grep -c v_writelane /tmp/fn.s)"
done
