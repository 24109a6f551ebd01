#!/bin/bash
# Round 4: the per-Gaussian backward split over two waves (geometry | SH, DG_LIVE_SPLIT) -- parity, then a same-box A/B
# of the raster bench and the native step.
set -e
OUT=${1:-gpurun_out/r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_training.py \
    tests/test_gpu_trainer.py tests/test_gpu_fullsize.py -q -rA --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
bash tools/abn.sh "$OUT/ab" 3 ab/live_one.so ab/live_split.so
for v in live_one live_split; do
  DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
      > "$OUT/nat_$v.txt" 2>&1
done
