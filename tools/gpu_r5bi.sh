#!/bin/bash
# where the (non-temporal) zero fill goes in the replay: HEAD (after the replay, first 3/4 of the launch order), at
# each wave's start (DG_BWD_FILL_EARLY), all waves (FRAC4=4), first half (FRAC4=2); kernel traces, two orders
OUT=${1:-gpurun_out/r5bi}
mkdir -p "$OUT"
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/early.so ablibs/all4.so ablibs/half.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/half.so ablibs/all4.so ablibs/early.so ablibs/base.so
