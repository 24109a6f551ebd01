#!/bin/bash
# per-phase times of the other workloads: 1e6 at 4K, 5e6 at 1080p
OUT=${1:-gpurun_out/r5x}
mkdir -p "$OUT"
B="--no-sweep --no-admm --no-train-step --no-cpu-baseline --steps 20 --warmup 4"
timeout -k 10 300 python bench.py $B --width 3840 --height 2160 > "$OUT/4k.json" 2> "$OUT/4k.err" || exit $?
timeout -k 10 300 python bench.py $B --gaussians 5000000 > "$OUT/5e6.json" 2> "$OUT/5e6.err" || exit $?
