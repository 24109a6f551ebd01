#!/bin/bash
# capacity contexts + torch-exact quaternion norm: the trainer / ADMM / activation tests, the first-step probe, then the
# config-5-shaped 8-rank rehearsal (rank 0 vs the sequential baseline, bit for bit?)
OUT=${1:-gpurun_out/r5n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_activations.py \
    tests/test_gpu_trainer_options.py tests/test_gpu_admm_run.py tests/test_gpu_admm_dist.py tests/test_gpu_raster.py \
    > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/first_step_probe.py > "$OUT/first_step.log" 2>&1
bash tools/gpu_r5k.sh "$OUT/k"
