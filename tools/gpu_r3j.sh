set -e
OUT=gpurun_out/r3j; mkdir -p $OUT/ab $OUT/ts
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/n9.so ab/n9_full.so
for i in 1 2; do for lib in n7 n9; do
  DOGS_HIP_LIB=ab/$lib.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/$lib.$i.log 2>&1
done; done
DOGS_HIP_LIB=ab/n9.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
