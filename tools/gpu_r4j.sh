#!/bin/bash
# Round 4: kernel timelines of one native and one autograd-route training step (bench.py's TrainStep).
set -e
OUT=${1:-gpurun_out/r4j}
mkdir -p "$OUT"
ROUTES=folded TB_ARGS="--bench-native" bash tools/train_timeline.sh "$OUT/native"
python tools/train_timeline.py "$OUT/native" > "$OUT/native_timeline.txt" 2>&1
ROUTES=folded TB_ARGS="--bench-autograd" bash tools/train_timeline.sh "$OUT/autograd"
python tools/train_timeline.py "$OUT/autograd" > "$OUT/autograd_timeline.txt" 2>&1
find "$OUT" -name "*kernel_trace.csv" -delete
