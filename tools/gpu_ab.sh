#!/bin/bash
# GPU step of a binning/kernel change: raster + full-size parity tests on the in-tree library, then an interleaved
# same-box A/B of the libraries given (tools/abn.sh), then a kernel trace of the in-tree build.
# usage: tools/gpu_ab.sh OUTDIR ROUNDS LIB1 [LIB2 ...]
set -e
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
DOGS_HIP_LIB=${TEST_LIB:-} timeout -k 10 500 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_fullsize.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
bash tools/abn.sh "$OUT/ab" "$R" "$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-train-step --no-reference-k --no-admm > "$OUT/trace.log" 2>&1
