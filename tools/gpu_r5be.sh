#!/bin/bash
# timing only: the backward without any zero fill of the gradient outputs against HEAD; build the variant first:
#   tools/build_variant.sh ablibs/nozero.so -DDG_NO_ZERO_FILL; cp dogs_amd/_lib/libdogs_hip.so ablibs/base.so
OUT=${1:-gpurun_out/r5be}
mkdir -p "$OUT"
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/nozero.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/nozero.so ablibs/base.so
