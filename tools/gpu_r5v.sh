#!/bin/bash
# live list with the Gaussian index: raster / trainer parity tests, bench phases, kernel trace of the bench
OUT=${1:-gpurun_out/r5v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_raster.py \
    tests/test_gpu_trainer_options.py tests/test_gpu_fullsize.py > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py \
    --no-cpu-baseline --no-admm --no-train-step --no-sweep --no-reference-k --steps 40 > "$OUT/kt.log" 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-admm --no-sweep > "$OUT/bench.json" 2> "$OUT/bench.err"
