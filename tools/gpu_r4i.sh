#!/bin/bash
# Round 4: row_prod (the scale regulariser without prod_backward's host read) -- parity, then the autograd route's time.
set -e
OUT=${1:-gpurun_out/r4i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py -q -rA --timeout 250 --timeout-method thread -k row_prod \
    > "$OUT/tests.log" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/native_100.txt" 2>&1
timeout -k 10 300 python tools/autograd_prof.py --steps 20 > "$OUT/autograd_prof.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_admm.py tests/test_gpu_trainer_options.py \
    -q -rA --timeout 300 --timeout-method thread > "$OUT/tests2.log" 2>&1 || true
