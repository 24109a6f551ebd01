#!/bin/bash
# timing only: the backward without any zero fill of the gradient outputs (DG_NO_ZERO_FILL) against HEAD
OUT=${1:-gpurun_out/r5be}
mkdir -p "$OUT"
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/nozero.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/nozero.so ablibs/base.so
