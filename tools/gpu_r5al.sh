#!/bin/bash
# kernel-level A/B of library builds at a fixed phase-1 capacity (DOGS_PREFIX_PER_TILE), kernel trace per build
# usage: tools/gpu_r5al.sh OUTDIR LIB...
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp DOGS_PREFIX_PER_TILE=${DOGS_PREFIX_PER_TILE:-448}
for lib in "$@"; do
  v=$(basename "$lib" .so)
  DOGS_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- \
      python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-train-step --no-admm --no-sweep --no-reference-k \
      > "$OUT/$v.log" 2>&1 || exit $?
done
