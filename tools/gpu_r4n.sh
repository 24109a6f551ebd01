#!/bin/bash
# Round 4: the whole -m gpu suite + smoke + default bench on the tree with the bucketed TensorArena and the cheaper
# stream / device lookups, both training routes, then the 4-rank gloo rehearsal of bench.py --gpus 4 on the shared GPU
# (2 x 2 ADMM split through admm_run).
set -e
OUT=${1:-gpurun_out/r4n}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_suite.sh "$OUT"
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/native_100.txt" 2>&1
( while true; do date +%T >> "$OUT/heartbeat4"; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 700 python bench.py --gpus 4 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench4.json" 2> "$OUT/bench4.err"
