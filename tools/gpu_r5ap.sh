#!/bin/bash
# DPP wave scans / reductions (binning walk, in-wave sorts, max contributors): parity with the new build, then
# kernel traces of the HEAD build and the new one, interleaved twice
OUT=${1:-gpurun_out/r5ap}
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=$PWD/ablibs/dpp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py > "$OUT/tests.log" 2>&1 || exit $?
bash tools/gpu_r5al.sh "$OUT/a" ablibs/base.so ablibs/dpp.so || exit $?
bash tools/gpu_r5al.sh "$OUT/b" ablibs/base.so ablibs/dpp.so
