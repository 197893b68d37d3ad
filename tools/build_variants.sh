#!/bin/bash
# Build diagnostic variants of libdgplace.so with extra -D flags (parallel), into
# tools/_var/lib_<name>.so; pick one at run time with DGP_LIB=<path>.
# usage: tools/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=2 -DBAR" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_var
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared -mllvm -amdgpu-lower-module-lds-strategy=module $flags \
    -o tools/_var/lib_$name.so distributed_amd/csrc/dgplace.hip 2> tools/_var/$name.err &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la tools/_var/*.so
