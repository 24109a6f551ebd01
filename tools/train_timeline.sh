#!/bin/bash
# Kernel traces of the native training step (tools/trainer_bench.py) for each update route of dg_train_step.
# usage: tools/train_timeline.sh OUTDIR   -- then: python tools/train_timeline.py OUTDIR
set -e
OUT=$1
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p "$OUT"
for route in ${ROUTES:-unfused folded}; do
  if [ "$route" = unfused ]; then export DG_TRAIN_UNFUSED=1; else unset DG_TRAIN_UNFUSED; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$route" -o run -- python3 "$ROOT/tools/trainer_bench.py" --steps 20 $TB_ARGS > "$OUT/$route.log" 2>&1
done
