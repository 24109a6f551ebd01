#!/bin/bash
# per-phase times and kernel traces of the other workloads (1e5 at 1080p, the sparse 1080p scene)
OUT=${1:-gpurun_out/r5t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --gaussians 100000 --no-sweep --no-admm --no-train-step --no-cpu-baseline \
    > "$OUT/b1e5.json" 2> "$OUT/b1e5.err" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt1e5" -o run -- python3 bench.py \
    --gaussians 100000 --no-cpu-baseline --no-admm --no-train-step --no-sweep --no-reference-k --steps 40 \
    > "$OUT/kt1e5.log" 2>&1 || exit $?
