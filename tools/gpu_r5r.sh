#!/bin/bash
# drop-in route glue: SSIM mean Function, L1 mean in one launch, unmaterialised raster gradients, row_prod stamps --
# aux / activation / trainer tests, the first-step probe, the autograd route's kernel trace, the bench's train leg
OUT=${1:-gpurun_out/r5r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_aux.py \
    tests/test_gpu_activations.py tests/test_gpu_trainer_options.py tests/test_gpu_trainer.py tests/test_gpu_admm.py \
    > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/first_step_probe.py > "$OUT/first_step.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ag" -o run -- python3 tools/autograd_host.py \
    --steps 40 > "$OUT/ag.log" 2>&1 || exit $?
python tools/step_gaps.py "$OUT/ag" > "$OUT/gaps.txt" 2>&1
timeout -k 10 300 python bench.py --no-sweep --no-admm --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
