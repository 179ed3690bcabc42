#!/bin/bash
# Build libcgamd.so with extra compile definitions into computer-graphics_amd/_build_<name>/
# (A/B experiments only; select it with CGAMD_LIB).  Usage: build_variant.sh NAME -DFOO ...
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/computer-graphics_amd/_build_$NAME
mkdir -p "$OUT"
cd "$ROOT/computer-graphics_amd"
objs=()
for f in csrc/*.hip; do
  o=$OUT/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -Wno-unused-function "$@" -c -o "$o" "$f" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libcgamd.so" "${objs[@]}"
echo "$OUT/libcgamd.so"
