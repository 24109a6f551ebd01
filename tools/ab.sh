#!/bin/bash
# Same-box A/B of two library builds: alternate A, B, A, B bench runs (each under its own timeout).
# usage: tools/ab.sh LIB_A LIB_B OUTDIR
set -e
A=$1; B=$2; OUT=${3:-gpurun_out/ab}
mkdir -p "$OUT"
for i in 1 2; do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    DOGS_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step > "$OUT/$v$i.log" 2>&1
  done
done
