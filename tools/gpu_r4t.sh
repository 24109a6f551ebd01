#!/bin/bash
# Round 4: the one-launch binning offsets for up to 262144 waves (5e6 Gaussians: 78k waves took the multi-launch scan)
# -- same-box A/B at 5e6.
set -e
OUT=${1:-gpurun_out/r4t}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-step --no-admm --n 5000000"
for r in 1 2 3; do
  for v in offs64k offs256k; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 $B > "$OUT/$v.$r.log" 2>&1
  done
done
