#!/bin/bash
# Round 4: interleaved Horner chains in the SSIM window sums (no s_nop before the DPP adds) -- A/B against the
# one-chain-per-sum build, then parity.
set -e
OUT=${1:-gpurun_out/r4k}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in ssim_horner ssim_inter; do
    echo "== $v" >> "$OUT/ssim_ab.txt"
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 120 python tools/ssim_bench.py 100 >> "$OUT/ssim_ab.txt" 2>&1
  done
done
for v in ssim_horner ssim_inter; do
  DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
      > "$OUT/train_$v.txt" 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_boundary.py tests/test_gpu_training.py tests/test_gpu_trainer.py -q -rA \
    --timeout 250 --timeout-method thread > "$OUT/tests.log" 2>&1
