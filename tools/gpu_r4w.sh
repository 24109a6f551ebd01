#!/bin/bash
# Round 4: the side-stream SH update forked before the main update (DG_SH_FORK_EARLY) -- overlap parity tests, then a
# same-box A/B of the native step (and its kernel timeline).
set -e
OUT=${1:-gpurun_out/r4w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_trainer.py tests/test_gpu_admm.py \
    tests/test_gpu_trainer_options.py -q -rA --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
for r in 1 2 3; do
  for v in fork_late fork_early; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
        > "$OUT/nat_$v.$r.txt" 2>&1
  done
done
ROUTES=folded TB_ARGS="--bench-native" bash tools/train_timeline.sh "$OUT/tl"
python tools/train_timeline.py "$OUT/tl" > "$OUT/native_timeline.txt" 2>&1
find "$OUT" -name "*kernel_trace.csv" -delete
