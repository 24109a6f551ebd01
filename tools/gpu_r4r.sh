#!/bin/bash
# Round 4: the long-list sort's tiles per block chosen from the phase-1 capacity -- 5e6 and 1e6 benches, the 5e6 parity
# tests.
set -e
OUT=${1:-gpurun_out/r4r}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-step --no-admm"
timeout -k 10 300 $B --n 5000000 > "$OUT/n5e6_1080p.log" 2>&1
timeout -k 10 300 $B > "$OUT/n1e6_1080p.log" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_raster.py -q -rA --timeout 500 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
