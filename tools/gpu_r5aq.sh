#!/bin/bash
# timing only: the phase-1 render without its in-wave radix passes (wrong order, DG_DSORT_NOSORT) vs HEAD
OUT=${1:-gpurun_out/r5aq}
mkdir -p "$OUT"
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/nosort.so
