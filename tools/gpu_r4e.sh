#!/bin/bash
# Round 4: the tests changed since the last suite run, the default bench (ADMM leg on dogs_amd.admm_run), the 2-rank
# gloo rehearsal, then the kernel trace + instruction-mix and HBM-traffic PMC passes of the bench workload.
# usage: tools/gpu_r4e.sh OUTDIR [traffic]   -- every GPU step under its own timeout; stops at the first failure
set -e
OUT=${1:-gpurun_out/r4e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm_run.py tests/test_gpu_trainer_options.py \
    tests/test_gpu_trainer.py -v -rA --timeout 500 --timeout-method thread > "$OUT/tests.log" 2>&1 || true
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 4 \
    --no-cpu-baseline --no-train-step > "$OUT/bench2.json" 2> "$OUT/bench2.err"
bash tools/profile.sh "$OUT/imix" pmc tools/pmc_imix.txt
python3 tools/imix.py "$OUT/imix" > "$OUT/imix.txt" 2>&1
cp "$OUT"/imix/trace/*kernel_stats.csv "$OUT/" 2>/dev/null || true
if [ "$2" = "traffic" ]; then
  bash tools/profile.sh "$OUT/prof" pmc
  python3 tools/pmc_traffic.py "$OUT/prof" 1000000 1920 1080 > "$OUT/pmc_traffic.log" 2>&1
  cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
  python3 tools/pmc_summary.py "$OUT/prof" > "$OUT/pmc_summary.txt" 2>&1
fi
rm -rf "$OUT"/imix/pmc* "$OUT"/imix/trace/*kernel_trace.csv "$OUT"/prof/pmc* "$OUT"/prof/trace/*kernel_trace.csv
