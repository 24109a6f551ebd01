#!/bin/bash
# round-5 evidence on the final tree: the whole -m gpu suite, smoke, the default bench line, its kernel trace, the 2-rank
# gloo rehearsal, then the PMC passes (tools/profile.sh) and the per-phase traffic table (profiles/pmc_traffic.json)
OUT=${1:-gpurun_out/r5u}
bash tools/gpu_r5i.sh "$OUT" || exit $?
bash tools/profile.sh "$OUT/prof" pmc || exit $?
python tools/pmc_traffic.py "$OUT/prof" 1000000 1920 1080 > "$OUT/pmc_traffic.log" 2>&1
python tools/pmc_summary.py "$OUT/prof" > "$OUT/pmc_summary.txt" 2>&1 || true
