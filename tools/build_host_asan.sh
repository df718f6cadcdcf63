#!/bin/bash
# Host-side AddressSanitizer build of the native code + the C-ABI driver tools/host_asan_selftest.cpp.
# Host code only: each -fsanitize= sits directly after -Xarch_host, the gfx950 code objects are built as usual.
# Output: tools/bin/host_asan_selftest (run it on a GPU box with ASAN_OPTIONS=verify_asan_link_order=0).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/bin
OBJ=$OUT/asan_obj
ROCM=${ROCM_PATH:-/opt/rocm}
mkdir -p "$OBJ"
FLAGS=(--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Wno-unused-variable -Wno-unused-function
       -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer)
pids=()
for src in "$ROOT"/csrc/*.hip "$ROOT"/csrc/comm/rccl_comm.cpp "$ROOT"/tools/host_asan_selftest.cpp; do
  o=$OBJ/$(basename "$src").o
  x=(); [[ $src == *.cpp ]] && x=(-x hip)
  "$ROCM/bin/hipcc" "${FLAGS[@]}" "${x[@]}" -c "$src" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
"$ROCM/bin/hipcc" --offload-arch=gfx950 -Xarch_host -fsanitize=address -o "$OUT/host_asan_selftest" "$OBJ"/*.o \
  -L"$ROCM/lib" -lrccl -Wl,-rpath,"$ROCM/lib"
echo "built $OUT/host_asan_selftest"
