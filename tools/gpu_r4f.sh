#!/bin/bash
# Round 4: SSIM Horner-form horizontal pass -- parity tests on the in-tree build, the SSIM kernels and the native train
# step of both variants interleaved (ab/ssim_horner.so, ab/ssim_tapfma.so), then the HBM-traffic PMC passes.
set -e
OUT=${1:-gpurun_out/r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_admm.py tests/test_gpu_training.py \
    tests/test_gpu_admm_run.py -q -rA --timeout 500 --timeout-method thread > "$OUT/tests.log" 2>&1 || true
for r in 1 2 3; do
  for v in ssim_horner ssim_tapfma ssim_pf4 ssim_pf6 ssim_r16 ssim_r16pf4; do
    echo "== $v" >> "$OUT/ssim_ab.txt"
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 120 python tools/ssim_bench.py 100 >> "$OUT/ssim_ab.txt" 2>&1
  done
  for v in ssim_horner ssim_tapfma; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 200 \
        > "$OUT/train_$v.$r.txt" 2>&1
  done
done
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 200 > "$OUT/train_autograd.txt" 2>&1
timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 --cprofile > "$OUT/train_autograd_cprof.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/agtrace" -o ag -- python3 tools/trainer_bench.py \
    --bench-autograd --steps 50 > "$OUT/agtrace.log" 2>&1
find "$OUT/agtrace" -name "*kernel_stats.csv" -exec cp {} "$OUT/autograd_kernel_stats.csv" \; || true
rm -rf "$OUT/agtrace"
bash tools/profile.sh "$OUT/prof" pmc
python3 tools/pmc_traffic.py "$OUT/prof" 1000000 1920 1080 > "$OUT/pmc_traffic.log" 2>&1
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
python3 tools/pmc_summary.py "$OUT/prof" > "$OUT/pmc_summary.txt" 2>&1
cp "$OUT"/prof/trace/*kernel_stats.csv "$OUT/" 2>/dev/null || true
rm -rf "$OUT"/prof/pmc* "$OUT"/prof/trace/*kernel_trace.csv
