#!/bin/bash
# the forward's one-select commit: raster parity (+ full sizes), the fixed tests, bench, autograd host phases
OUT=${1:-gpurun_out/r5c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_raster.py \
    tests/test_gpu_fullsize.py tests/test_gpu_boundary.py "tests/test_gpu_admm_run.py::test_ranks_match_sequential_run" \
    tests/test_gpu_trainer_options.py > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-admm > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 200 python tools/autograd_host.py > "$OUT/autograd_host.log" 2>&1
