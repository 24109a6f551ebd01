#!/bin/bash
# Kernel-trace stats + separate PMC passes of the bench workload (run on the GPU box from the repo root).
# usage: [BENCH_ARGS="--width 3840 --height 2160"] tools/profile.sh OUTDIR [pmc [COUNTERS_FILE]]   -- each GPU step
# under its own timeout; stops at the first failure (COUNTERS_FILE: one "pmc: ..." pass per line, default
# tools/pmc_counters.txt; BENCH_ARGS: the workload, default the bench's 1e6 at 1080p)
set -e
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-train-step --no-reference-k --no-admm --no-sweep ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.log" 2>&1
if [ "$2" = "pmc" ]; then
  i=0
  while read -r line; do
    case "$line" in pmc:*) ;; *) continue ;; esac
    i=$((i+1))
    ctrs=${line#pmc: }
    timeout -k 10 300 rocprofv3 --pmc $ctrs -d "$OUT/pmc$i" -o run -- python3 $BENCH > "$OUT/pmc$i.log" 2>&1
  done < "${3:-$ROOT/tools/pmc_counters.txt}"
fi
