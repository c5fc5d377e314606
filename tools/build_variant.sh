#!/bin/bash
# Build a variant of the codec library for an A/B run: the kernel sources
# compiled with extra -D flags (experiment macros under development), linked
# with the in-tree host objects, into ab/lib_<name>.so. Bench it with
# REDSET_HIP_LIBRARY=$PWD/ab/lib_<name>.so on the GPU box.
# usage: tools/build_variant.sh <name> "<-D flags>"
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1 flags=${2:-}
obj=ab/obj_$name
mkdir -p "$obj"
pids=()
for f in redset_amd/csrc/codec_kernels.hip redset_amd/csrc/codec_sets_*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Iinclude \
    $flags -c "$f" -o "$obj/$(basename "${f%.hip}").o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
host=(redset_amd/build/redset_hip.o redset_amd/build/gf256.o redset_amd/build/stripe_map.o
      redset_amd/build/stream_pipeline.o redset_amd/build/sharded.o redset_amd/build/transport_rccl.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/lib_$name.so" "$obj"/*.o "${host[@]}" -lpthread -ldl \
  -Wl,-rpath,/opt/rocm/lib
rm -rf "$obj"
echo "ab/lib_$name.so"
