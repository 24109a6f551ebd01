#!/bin/bash
# kernel trace of the 5e6-Gaussian 1080p workload (the sweep's 5e6 case as the main loop)
OUT=${1:-gpurun_out/r5av}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --n 5000000 \
    --steps 16 --warmup 8 --no-cpu-baseline --no-train-step --no-admm --no-sweep --no-reference-k > "$OUT/kt.log" 2>&1
