#!/bin/bash
# A training-step change: the trainer / training / ADMM / option parity tests on the in-tree build, then a same-box A/B
# of the given builds on the native step (tools/gpu_ab_train.sh) and a kernel timeline of the in-tree step.
# usage: tools/gpu_ab_train_tests.sh OUTDIR ROUNDS LIB1 [LIB2 ...]
set -e
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_trainer.py tests/test_gpu_admm.py \
    tests/test_gpu_trainer_options.py tests/test_gpu_optim.py tests/test_gpu_admm_run.py -q -rA --timeout 600 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
bash tools/gpu_ab_train.sh "$OUT" "$R" "$@"
ROUTES=folded TB_ARGS="--bench-native" bash tools/train_timeline.sh "$OUT/tl"
python tools/train_timeline.py "$OUT/tl" > "$OUT/native_timeline.txt" 2>&1
find "$OUT" -name "*kernel_trace.csv" -delete
