#!/bin/bash
# Instruction statistics of the stream roles' out-of-line functions in the current sources.
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
  -mllvm -amdgpu-lower-module-lds-strategy=module --offload-device-only $@ -o /tmp/dev.co /root/repo/distributed_amd/csrc/dgplace.hip 2>/dev/null
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/dev.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/dev950.o
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 /tmp/dev950.o > /tmp/dev.s
for f in entry_exeILb1EEEvv \
         exe_run_entryILb1EEEbix15HIP_vector_typeIjLj4EE build_desc_g_entryEx build_desc_seq_entryEx \
         entry_regILb1EEEvv entry_wlkILb1EEEvv entry_stageILi0EEEvv entry_stageILi1EEEvv; do
  a=$(grep -n "${f}>:" /tmp/dev.s | head -1 | cut -d: -f1)
  [ -z "$a" ] && { echo "$f: not found"; continue; }
  b=$(awk -v s=$a 'NR>s && />:$/ {print NR; exit}' /tmp/dev.s)
  sed -n "${a},${b}p" /tmp/dev.s > /tmp/fn_$f.s
  n=$(wc -l < /tmp/fn_$f.s)
  body=$(grep -n "scratch_" /tmp/fn_$f.s | awk -F: -v n=$n '$1>80 && $1<n-120' | wc -l)
  echo "$f lines $n scratch $(grep -c scratch_ /tmp/fn_$f.s) (body $body) readlane $(grep -c v_readlane /tmp/fn_$f.s) writelane $(grep -c v_writelane /tmp/fn_$f.s)"
done
