#!/bin/bash
# the phase entry's stages (DOGS_ENTRY_TIMING=1) in the bench-sized ADMM rehearsal: 2 and 4 gloo ranks at 1080p
OUT=${1:-gpurun_out/r5ad}
mkdir -p "$OUT"
export TMPDIR=/tmp DOGS_ENTRY_TIMING=1 DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1
for np in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node $np --master-addr 127.0.0.1 \
      --master-port 29534 tools/admm_rehearsal.py --points 1000000 --admm-pre 200 --admm-interval 200 \
      > "$OUT/r$np.json" 2> "$OUT/r$np.err" || exit $?
done
