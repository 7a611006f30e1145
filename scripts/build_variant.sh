#!/usr/bin/env bash
# Builds an A/B variant of libcfdsim.so: recompiles the named translation
# units with extra -D flags and links them with the other objects of the
# in-tree build (cfd-simulations_amd/csrc/build).  Output: build_<name>/libcfdsim.so
# usage: scripts/build_variant.sh NAME "HIPCC FLAGS" unit.hip [unit.hip ...]
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2; shift 2
src=cfd-simulations_amd/csrc
out=build_$name
mkdir -p "$out"
objs=()
for o in "$src"/build/*.o; do
  b=$(basename "$o" .o)
  keep=1
  for u in "$@"; do [ "$b" = "$(basename "$u" .hip)" ] && keep=0; done
  [ $keep = 1 ] && objs+=("$o")
done
for u in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result \
    $flags -I "$src" -c "$src/$u" -o "$out/$(basename "$u" .hip).o" &
done
wait
for u in "$@"; do objs+=("$out/$(basename "$u" .hip).o"); done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/libcfdsim.so" "${objs[@]}" -L/opt/rocm/lib -lrccl
echo "built $out/libcfdsim.so"
