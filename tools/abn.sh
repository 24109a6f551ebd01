#!/bin/bash
# Same-box comparison of several library builds: R rounds of one bench run per library, interleaved.
# usage: tools/abn.sh OUTDIR ROUNDS LIB1 [LIB2 ...]   (each run under its own timeout; stops at the first failure)
set -e
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
    DOGS_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step --no-admm --no-reference-k --no-sweep > "$OUT/$v.$i.log" 2>&1
  done
done
