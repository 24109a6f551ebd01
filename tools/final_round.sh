#!/bin/bash
# Round-end evidence on one GPU box, from the repo root: the whole GPU suite, smoke, the kernel trace and the separate
# PMC passes of the bench workload (tools/profile.sh), the per-phase traffic table the bench reads
# (tools/pmc_traffic.py -> profiles/pmc_traffic.json, copied into OUT), then the default bench line.
# usage: tools/final_round.sh OUTDIR   -- each GPU step under its own timeout; stops at the first failure
set -e
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
bash tools/profile.sh "$OUT/prof" pmc
python3 tools/pmc_traffic.py "$OUT/prof" 1000000 1920 1080 > "$OUT/pmc_traffic.log" 2>&1
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
python3 tools/pmc_summary.py "$OUT/prof" > "$OUT/pmc_summary.txt" 2>&1
# the raw per-dispatch counter dumps exceed gpurun's copy-back limit: keep the summaries and the trace statistics
cp "$OUT"/prof/trace/*kernel_stats.csv "$OUT/" 2>/dev/null || true
rm -rf "$OUT"/prof/pmc* "$OUT"/prof/trace/*kernel_trace.csv
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
