#!/bin/bash
OUT=${1:-gpurun_out/r5e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/mask_det_probe.py --block 1 > "$OUT/mask_det.log" 2>&1
timeout -k 10 200 python tools/trainer_bench.py --bench-autograd --steps 40 --cprofile --autograd-main-thread > "$OUT/cprof.log" 2>&1
