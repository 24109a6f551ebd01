#!/bin/bash
OUT=${1:-gpurun_out/r5l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/first_step_probe.py > "$OUT/first_step.log" 2>&1
bash tools/gpu_r5k.sh "$OUT/k"
