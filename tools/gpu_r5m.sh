#!/bin/bash
OUT=${1:-gpurun_out/r5m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/act_match_probe.py > "$OUT/act_match.log" 2>&1
bash tools/gpu_r5k.sh "$OUT/k"
