#!/bin/bash
# Round 4: the binning offsets by the count pass's last block (DG_BIN_TAIL) -- parity on the raster / trainer tests,
# then a same-box A/B of the raster bench and the native step.
set -e
OUT=${1:-gpurun_out/r4o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_streams.py \
    tests/test_gpu_fullsize.py tests/test_gpu_trainer.py tests/test_gpu_primitives.py -q -rA --timeout 600 \
    --timeout-method thread > "$OUT/tests.log" 2>&1
bash tools/abn.sh "$OUT/ab" 3 ab/tail_off.so ab/tail_on.so
for r in 1 2; do
  for v in tail_off tail_on; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
        > "$OUT/nat_$v.$r.txt" 2>&1
  done
done
