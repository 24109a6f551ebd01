#!/bin/bash
# gauss_sum: the segmented scan skipped for steps without a flagged record
OUT=${1:-gpurun_out/r5ar}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/sumskip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/sumskip.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/base.so ablibs/sumskip.so
