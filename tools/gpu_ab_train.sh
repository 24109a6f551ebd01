#!/bin/bash
# Same-box A/B of library builds on the training step: R rounds of tools/trainer_bench.py per library, interleaved
# (native step; AUTOGRAD=1 adds the autograd route), each run under its own timeout.
# usage: tools/gpu_ab_train.sh OUTDIR ROUNDS LIB1 [LIB2 ...]
set -e
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 "$R"); do
  for lib in "$@"; do
    v=$(basename "$lib" .so)
    DOGS_HIP_LIB=$lib timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/nat_$v.$i.txt" 2>&1
    if [ -n "$AUTOGRAD" ]; then
      DOGS_HIP_LIB=$lib timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 \
          > "$OUT/ag_$v.$i.txt" 2>&1
    fi
  done
done
