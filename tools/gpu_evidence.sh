#!/bin/bash
# Evidence of the committed tree: the whole -m gpu suite + smoke + default bench (tools/gpu_suite.sh),
# then the kernel-trace stats of the bench workload (tools/profile.sh, no counters).
set -e
OUT=${1:-gpurun_out/evidence}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_suite.sh "$OUT"
bash tools/profile.sh "$OUT/prof"
cp "$OUT"/prof/trace/*kernel_stats.csv "$OUT/" 2>/dev/null || true
rm -rf "$OUT"/prof/trace/*kernel_trace.csv
