#!/bin/bash
# the replay prologue with non-temporal per-pixel loads: bit-identity, parity, kernel traces
OUT=${1:-gpurun_out/r5bh}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base ntl; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 python -u tools/bitcmp.py "$OUT/bits_$v.json" > "$OUT/bits_$v.log" 2>&1 || exit $?
done
python tools/bitcmp.py --cmp "$OUT/bits_base.json" "$OUT/bits_ntl.json" > "$OUT/bitcmp.txt" 2>&1
DOGS_HIP_LIB=$PWD/ablibs/ntl.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/ntl.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/ntl.so ablibs/base.so
