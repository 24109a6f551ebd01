#!/bin/bash
# Round 4: dense long-list sorts at 5e6 -- a wave per tile + a 1024-block long sort (DG_DSORT_DENSE_SPLIT) vs the
# merged kernel at 4 tiles per block; then the 5e6 parity tests on the default build.
set -e
OUT=${1:-gpurun_out/r4s}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-step --no-admm --n 5000000"
for r in 1 2; do
  for v in dsort_tpb4 dsort_split; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 $B > "$OUT/$v.$r.log" 2>&1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -q -rA --timeout 500 --timeout-method thread \
    > "$OUT/tests.log" 2>&1
