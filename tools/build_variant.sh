#!/bin/bash
# Build a variant of the library with extra compile flags into abtest/<name>.so (for tools/ab_libs.sh)
# usage: tools/build_variant.sh <name> <flags...>
set -e
name=$1; shift
cd "$(dirname "$0")/../zk-research-implementations_amd"
d=/tmp/zkvar_$name; mkdir -p $d ../abtest
for f in zk_sumcheck gkr_circuit kzg blob; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c -o $d/$f.o csrc/$f.hip &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o ../abtest/$name.so $d/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built abtest/$name.so
