#!/bin/bash
# Tuning build of the kernel library (timing ablations with wrong results reachable: skipped epilogues / staging,
# pp-kernel variants 5-9): build/tuning/libedge_kernels.so, loaded with EDGE_KERNEL_LIB for A/B runs
# (tools/gemm_bench.py).  Never the production library.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/tuning
objs=()
for f in csrc/*.hip; do
  o=build/tuning/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DEDGE_TUNING_BUILD=1 -Wno-unused-variable \
    -Wno-unused-function -c $f -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/tuning/libedge_kernels.so "${objs[@]}"
echo build/tuning/libedge_kernels.so
