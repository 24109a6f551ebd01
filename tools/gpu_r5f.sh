#!/bin/bash
OUT=${1:-gpurun_out/r5f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/mask_conc_probe.py > "$OUT/mask_conc.log" 2>&1
