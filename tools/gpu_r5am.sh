#!/bin/bash
# binning offsets, one-round DPP scan: raster parity with the new build, then kernel traces of old/new interleaved
OUT=${1:-gpurun_out/r5am}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/bo_new3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/bo_old.so ablibs/bo_new3.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/bo_old.so ablibs/bo_new3.so
