#!/bin/bash
# the replay's zero fill with non-temporal stores: bit-identity at 1e6 against HEAD, parity, kernel traces
OUT=${1:-gpurun_out/r5bf}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base nt; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 python -u tools/bitcmp.py "$OUT/bits_$v.json" > "$OUT/bits_$v.log" 2>&1 || exit $?
done
python tools/bitcmp.py --cmp "$OUT/bits_base.json" "$OUT/bits_nt.json" > "$OUT/bitcmp.txt" 2>&1
DOGS_HIP_LIB=$PWD/ablibs/nt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/nt.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/nt.so ablibs/base.so
