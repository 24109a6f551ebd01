#!/bin/bash
# config-5-shaped rehearsal: 8 gloo ranks sharing the one GPU, 4K views, ~2.5e6 Gaussians per block, a 4 x 2 Grid2D
# ADMM split (pre-phase with densification, phase entry with the all-gather of the fused model, one round), then the
# sequential baseline on rank 0.  Times measure the shared GPU and gloo, not RCCL; the point is the shapes and sizes.
OUT=${1:-gpurun_out/r5k}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat"; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 900 python bench.py --gpus 8 --steps 4 --warmup 2 \
    --gaussians 2500000 --width 3840 --height 2160 --admm-pre 100 --admm-interval 100 --admm-rounds 1 --no-cpu-baseline \
    --no-train-step --no-reference-k > "$OUT/bench8.json" 2> "$OUT/bench8.err"
echo "rc=$?" >> "$OUT/bench8.err"
