set -e
OUT=gpurun_out/r3f; mkdir -p $OUT/ab $OUT/ts
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
DOGS_HIP_LIB=ab/rowwalk.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/rowwalk_tests.log 2>&1 || { echo "rowwalk tests rc=$?" >> $OUT/rowwalk_tests.log; exit 0; }
for lib in ab/new4.so ab/ssim1.so ab/ssim2w3.so ab/new4.so ab/ssim1.so ab/ssim2w3.so; do
  DOGS_HIP_LIB=$lib timeout -k 10 120 python tools/ssim_bench.py 200 >> $OUT/ssim_bench.txt 2>&1
done
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/new4.so ab/new4_2l.so ab/new4_mc.so ab/rowwalk.so
for i in 1 2; do for lib in ab/new4.so ab/ssim1.so; do
  DOGS_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/$(basename $lib .so).$i.log 2>&1
done; done
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
