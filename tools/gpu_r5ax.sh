#!/bin/bash
# ranges scan at 16 vs 32 items per thread, 5e6 Gaussians (5 vs 3 rounds): parity of the 32-item build, kernel traces
OUT=${1:-gpurun_out/r5ax}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/bo32.so timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_raster.py -k "many_binning or bitexact" > "$OUT/tests.log" 2>&1 || exit $?
for v in bo2 bo32 bo2 bo32; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/k5_$v$RANDOM" -o run -- \
      python3 bench.py --n 5000000 --steps 8 --warmup 4 --no-cpu-baseline --no-train-step --no-admm --no-sweep \
      --no-reference-k > "$OUT/k5_$v.log" 2>&1 || exit $?
done
