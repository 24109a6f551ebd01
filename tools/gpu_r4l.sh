#!/bin/bash
# Round 4: the counters published by k_depth_cut (the forward's host wait ends before the binning) -- the whole
# -m gpu suite + smoke + default bench, then both training routes.
set -e
OUT=${1:-gpurun_out/r4l}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_suite.sh "$OUT"
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/native_100.txt" 2>&1
