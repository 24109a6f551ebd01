#!/bin/bash
# Kernel-trace stats of the bench workload for several library builds (same box).
# usage: tools/kprof.sh OUTDIR LIB1 [LIB2 ...]   -- each run under its own timeout; stops at the first failure
set -e
OUT=$1; shift
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p "$OUT"
for lib in "$@"; do
  v=$(basename "$lib" .so)
  DOGS_HIP_LIB=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-step --no-admm --no-reference-k > "$OUT/$v.log" 2>&1
done
