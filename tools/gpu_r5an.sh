#!/bin/bash
# depth histogram block size: kernel traces of base / 32 / 64 items per thread, interleaved twice
OUT=${1:-gpurun_out/r5an}
mkdir -p "$OUT"
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/dh32.so ablibs/dh64.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/base.so ablibs/dh32.so ablibs/dh64.so
