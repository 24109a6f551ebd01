#!/bin/bash
# Round 4: the 4-rank gloo rehearsal of bench.py --gpus 4 on the shared GPU (2 x 2 ADMM split through admm_run), the
# raster/boundary/stream tests on the bucketed TensorArena, and the autograd route's time.
set -e
OUT=${1:-gpurun_out/r4n}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat"; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_streams.py \
    -q -rA --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 700 python bench.py --gpus 4 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench4.json" 2> "$OUT/bench4.err"
