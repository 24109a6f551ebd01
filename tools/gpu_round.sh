#!/bin/bash
# One GPU call per round: the counter list, the whole -m gpu suite + smoke + default bench (tools/gpu_suite.sh), the
# 2-rank gloo rehearsal of bench.py --gpus 2 on the shared GPU, then an interleaved same-box A/B of ab/*.so.
# usage: tools/gpu_round.sh OUTDIR [ROUNDS]   -- every GPU step under its own timeout; stops at the first failure
set -e
OUT=${1:-gpurun_out/r4}; R=${2:-3}
mkdir -p "$OUT"
export TMPDIR=/tmp
(timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true)
bash tools/gpu_suite.sh "$OUT"
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench2.json" 2> "$OUT/bench2.err"
if ls ab/*.so > /dev/null 2>&1; then bash tools/abn.sh "$OUT/ab" "$R" ab/*.so; fi
