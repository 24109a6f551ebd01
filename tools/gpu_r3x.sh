set -e
OUT=gpurun_out/r3x; mkdir -p $OUT/ab $OUT/cap
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_fullsize.py tests/test_gpu_boundary.py tests/test_gpu_aux.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/base.so ab/skip0.so
for c in 0 320 384 512; do
  DOGS_PREFIX_PER_TILE=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step --no-admm --no-reference-k > $OUT/cap/c$c.log 2>&1
done
bash tools/kprof.sh $OUT/kp ab/skip0.so
