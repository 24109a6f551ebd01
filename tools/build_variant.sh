#!/bin/bash
# Build a variant of libdogs_hip.so with extra compile flags into OUT (for same-box A/B timing experiments).
# usage: [SRC=dir] tools/build_variant.sh OUT.so [-DFLAG ...]
#   SRC: a directory holding the library's sources (default dogs_amd/csrc), e.g. a copy with one file swapped for an
#   older version; the source list and flags are dogs_amd/build.py's.
set -e
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=${SRC:-$ROOT/dogs_amd/csrc}
TMP=$(mktemp -d)
read -r -a SOURCES <<< "$(cd "$ROOT" && python -c 'from dogs_amd.build import SOURCES; print(" ".join(SOURCES))')"
read -r -a FLAGS <<< "$(cd "$ROOT" && python -c 'from dogs_amd.build import FLAGS; print(" ".join(FLAGS))')"
pids=()
for s in "${SOURCES[@]}"; do
  hipcc "${FLAGS[@]}" "$@" -c "$SRC/$s" -o "$TMP/${s%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
hipcc -shared -fPIC --offload-arch=gfx950 "$TMP"/*.o -o "$OUT"
rm -rf "$TMP"
