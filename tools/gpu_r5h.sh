#!/bin/bash
# phase-2 segments: raster parity (+ full sizes), masked distributed run, then an interleaved A/B of segments on / off
OUT=${1:-gpurun_out/r5h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_raster.py \
    tests/test_gpu_fullsize.py tests/test_gpu_boundary.py tests/test_gpu_admm_run.py > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-admm --no-train-step --no-reference-k --no-sweep --steps 40 \
      > "$OUT/seg_$r.json" 2>/dev/null || exit $?
  DG_FWD2_NO_SEGMENTS=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-admm --no-train-step --no-reference-k \
      --no-sweep --steps 40 > "$OUT/noseg_$r.json" 2>/dev/null || exit $?
done
