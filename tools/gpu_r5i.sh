#!/bin/bash
# evidence run: whole -m gpu suite + smoke + default bench, the bench under a kernel trace, the 2-rank gloo rehearsal
OUT=${1:-gpurun_out/r5i}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_suite.sh "$OUT" || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py \
    --no-cpu-baseline --no-admm --no-train-step --no-sweep --no-reference-k --steps 40 > "$OUT/kt.log" 2>&1 || exit $?
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench2.json" 2> "$OUT/bench2.err"
