#!/bin/bash
# Round 4: the SSIM parity bar against the float64 value (Horner-form window sums), and the autograd route's host
# profile (torch.profiler op table; cProfile with the backward on the calling thread).
set -e
OUT=${1:-gpurun_out/r4h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_boundary.py -q -rA --timeout 250 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || true
timeout -k 10 300 python tools/autograd_prof.py --steps 20 > "$OUT/autograd_prof.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 --cprofile --autograd-main-thread \
    > "$OUT/autograd_cprof_main.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/native_100.txt" 2>&1
