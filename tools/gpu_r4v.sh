#!/bin/bash
# Round 4: final evidence of the committed tree (the whole -m gpu suite + smoke + default bench + kernel-trace stats,
# tools/gpu_r4final.sh), the autograd route's time, then the one-launch binning offsets A/B at 5e6 (tools/gpu_r4t.sh).
set -e
OUT=${1:-gpurun_out/r4v}
bash tools/gpu_r4final.sh "$OUT"
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 > "$OUT/autograd_100.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 > "$OUT/native_100.txt" 2>&1
bash tools/gpu_r4t.sh gpurun_out/r4t
