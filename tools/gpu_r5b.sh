#!/bin/bash
# determinism probe, then the whole -m gpu suite + smoke + default bench (tools/gpu_suite.sh), then the native trainer
# bench under a kernel trace (clean exit, csv stats)
OUT=${1:-gpurun_out/r5b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/det_probe.py > "$OUT/det_probe.log" 2>&1 || exit $?
bash tools/gpu_suite.sh "$OUT" || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kp" -o run -- python3 tools/trainer_bench.py \
    --bench-native --steps 40 > "$OUT/kp.log" 2>&1
echo "rocprof rc=$?" >> "$OUT/kp.log"
