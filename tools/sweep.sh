#!/bin/bash
# Bench sweep of the workloads SURVEY.md 8(d) names (N in {1e5, 1e6, 5e6} at 1080p; 800x800; 4K) plus a 2-rank
# rehearsal of the ADMM path on one GPU (gloo, shared device).  usage: tools/sweep.sh OUTDIR
set -e
OUT=${1:-gpurun_out/sweep}
mkdir -p "$OUT"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-step --no-admm"
timeout -k 10 300 $B --n 100000 > "$OUT/n1e5_1080p.log" 2>&1
timeout -k 10 300 $B --n 5000000 > "$OUT/n5e6_1080p.log" 2>&1
timeout -k 10 300 $B --n 100000 --width 800 --height 800 > "$OUT/n1e5_800.log" 2>&1
timeout -k 10 300 $B --n 1000000 --width 3840 --height 2160 > "$OUT/n1e6_4k.log" 2>&1
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
  --no-cpu-baseline --no-train-step --no-admm > "$OUT/n1e6_2rank_gloo.log" 2>&1
