#!/bin/bash
# one-launch ranges scan up to 262144 wave totals with the next round prefetched: parity (raster + full-size views at
# 5e6) with the new build, bit-identity at 5e6 against HEAD, kernel traces at 5e6 and 1e6 (base first, then reversed)
OUT=${1:-gpurun_out/r5aw}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/bo2.so timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_fullsize.py > "$OUT/tests.log" 2>&1 || exit $?
for v in base bo2; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 python -u tools/bitcmp.py "$OUT/bits_$v.json" --n 5000000 > "$OUT/bits_$v.log" 2>&1 || exit $?
done
python tools/bitcmp.py --cmp "$OUT/bits_base.json" "$OUT/bits_bo2.json" > "$OUT/bitcmp.txt" 2>&1
for v in base bo2; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/k5_$v" -o run -- \
      python3 bench.py --n 5000000 --steps 16 --warmup 8 --no-cpu-baseline --no-train-step --no-admm --no-sweep \
      --no-reference-k > "$OUT/k5_$v.log" 2>&1 || exit $?
done
bash tools/gpu_r5al.sh "$OUT/b" ablibs/bo2.so ablibs/base.so
