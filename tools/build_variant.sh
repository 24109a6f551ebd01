#!/bin/bash
# Build a variant of libdogs_hip.so with extra compile flags into OUT (for same-box A/B timing experiments).
# usage: tools/build_variant.sh OUT.so [-DFLAG ...]
set -e
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -munsafe-fp-atomics"
pids=()
for s in sortscan raster_fwd raster_bwd aux_kernels optim export loader blocksplit colmap capi; do
  hipcc $FLAGS "$@" -c "$ROOT/dogs_amd/csrc/$s.hip" -o "$TMP/$s.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
hipcc -shared -fPIC --offload-arch=gfx950 "$TMP"/*.o -o "$OUT"
rm -rf "$TMP"
