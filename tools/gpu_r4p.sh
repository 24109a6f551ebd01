#!/bin/bash
# Round 4: DG_BIN_TAIL with plain loads after the acquire fence -- A/B of the raster bench and the native step, then
# the raster parity tests.
set -e
OUT=${1:-gpurun_out/r4p}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/abn.sh "$OUT/ab" 3 ab/tail_off.so ab/tail_on.so
for v in tail_off tail_on; do
  DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
      > "$OUT/nat_$v.txt" 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_fullsize.py -q -rA --timeout 500 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
