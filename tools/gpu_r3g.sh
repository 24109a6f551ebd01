set -e
OUT=gpurun_out/r3g; mkdir -p $OUT/ab $OUT/ts
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
for lib in ab/new6.so ab/s_f1.so ab/s_b24.so ab/s_1col.so ab/new6.so ab/s_f1.so ab/s_b24.so ab/s_1col.so; do
  DOGS_HIP_LIB=$lib timeout -k 10 120 python tools/ssim_bench.py 200 >> $OUT/ssim_bench.txt 2>&1
done
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/new6.so ab/new6_mc.so
for i in 1 2; do for lib in ab/new6.so ab/s_f1.so ab/s_1col.so; do
  DOGS_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/$(basename $lib .so).$i.log 2>&1
done; done
timeout -k 10 300 python tools/replay_probe.py > $OUT/replay_probe.txt 2>&1
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
