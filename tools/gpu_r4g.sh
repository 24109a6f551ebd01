#!/bin/bash
# Round 4: the 4-rank gloo rehearsal of bench.py --gpus 4 on the shared GPU (2 x 2 ADMM split through admm_run), then
# the whole -m gpu suite + smoke + default bench of the final tree.
set -e
OUT=${1:-gpurun_out/r4g}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python bench.py --gpus 4 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench4.json" 2> "$OUT/bench4.err"
bash tools/gpu_suite.sh "$OUT"
