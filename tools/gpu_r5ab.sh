#!/bin/bash
# MatrixCity-shaped rehearsal at full per-block scale (BASELINE config 5: >= 5e6 Gaussians per block, 4K views) on the
# one-GPU box: 2 gloo ranks sharing the GPU, 13e6 points per block -- pre-phase with densification, the phase entry,
# ADMM rounds, then rank 0's sequential baseline, rank 0's block compared bit for bit (tools/admm_rehearsal.py: the
# bench's ADMM leg without its raster leg).  The 8-rank 2 x 4 split ran at 2.5e6 per rank in
# profiles/r05n_bench_8rank_gloo_shared_4k.json.
OUT=${1:-gpurun_out/r5ab}
PTS=${PTS:-13000000}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat"; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 ${TO:-850} python -m torch.distributed.run --nnodes 1 \
    --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29533 tools/admm_rehearsal.py --points "$PTS" \
    --width 3840 --height 2160 --admm-pre 100 --admm-interval 100 > "$OUT/rehearsal.json" 2> "$OUT/rehearsal.err"
