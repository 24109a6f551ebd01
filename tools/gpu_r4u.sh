#!/bin/bash
# Round 4: the cached Adam group tables -- optimizer / trainer / ADMM parity tests and the autograd route's time; then
# the one-launch binning offsets A/B at 5e6 (tools/gpu_r4t.sh).
set -e
OUT=${1:-gpurun_out/r4u}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_trainer.py tests/test_gpu_admm.py \
    tests/test_gpu_training.py -q -rA --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
bash tools/gpu_r4t.sh gpurun_out/r4t
