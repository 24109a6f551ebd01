#!/bin/bash
# packed 1 - alpha and dx in the forward and the replay: bit-identity against HEAD on the bench workload, parity tests,
# then kernel traces base / pk / pk5 (pk with the forward capped at 5 waves per SIMD), interleaved twice
OUT=${1:-gpurun_out/r5as}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base pk pk5; do
  DOGS_HIP_LIB=$PWD/ablibs/$v.so timeout -k 10 300 python -u tools/bitcmp.py "$OUT/bits_$v.json" > "$OUT/bits_$v.log" 2>&1 || exit $?
done
python tools/bitcmp.py --cmp "$OUT/bits_base.json" "$OUT/bits_pk.json" > "$OUT/bitcmp.txt" 2>&1
python tools/bitcmp.py --cmp "$OUT/bits_base.json" "$OUT/bits_pk5.json" >> "$OUT/bitcmp.txt" 2>&1
DOGS_HIP_LIB=$PWD/ablibs/pk.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/pk.so ablibs/pk5.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/pk5.so ablibs/pk.so ablibs/base.so
