#!/bin/bash
# round 5, first call: the changed / new GPU tests, then the native trainer bench under a kernel trace (clean exit?)
OUT=${1:-gpurun_out/r5a}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat"; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -v -rA --timeout 600 --timeout-method thread \
    tests/test_gpu_admm_run.py tests/test_gpu_trainer_options.py "tests/test_gpu_aux.py::test_fused_ssim_matches_oracle" \
    > "$OUT/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kp" -o run -- python3 tools/trainer_bench.py --bench-native --steps 40 \
    > "$OUT/kp.log" 2>&1
echo "rocprof rc=$?" >> "$OUT/kp.log"
