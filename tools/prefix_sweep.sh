#!/bin/bash
# Bench the phase-1 binning capacity per tile (DOGS_PREFIX_PER_TILE) on one box.
# usage: tools/prefix_sweep.sh OUTDIR CAP1 [CAP2 ...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
for c in "$@"; do
  DOGS_PREFIX_PER_TILE=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step > "$OUT/cap$c.log" 2>&1
done
