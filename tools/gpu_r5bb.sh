#!/bin/bash
# emission: key, record, count and wave base in one load round
# kernel traces at 1e6 (base first, then reversed)
OUT=${1:-gpurun_out/r5bb}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/emit1.so timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_fullsize.py tests/test_gpu_boundary.py > "$OUT/tests.log" 2>&1 || exit $?
for n in 1000000 5000000; do
  for v in base emit1; do
    DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 python -u tools/bitcmp.py "$OUT/bits_${v}_$n.json" --n $n > "$OUT/bits_${v}_$n.log" 2>&1 || exit $?
  done
  python tools/bitcmp.py --cmp "$OUT/bits_base_$n.json" "$OUT/bits_emit1_$n.json" >> "$OUT/bitcmp.txt" 2>&1
done
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/emit1.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/emit1.so ablibs/base.so
