#!/bin/bash
OUT=${1:-gpurun_out/r5d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/mask_det_probe.py > "$OUT/mask_det.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-admm > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 200 python tools/autograd_host.py > "$OUT/autograd_host.log" 2>&1
