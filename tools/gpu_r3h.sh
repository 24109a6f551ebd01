set -e
OUT=gpurun_out/r3h; mkdir -p $OUT/ab
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/n7.so ab/n7_mc.so
for lib in n7 n7_ac n7_noadam; do
  DOGS_HIP_LIB=ab/$lib.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt_$lib
  python3 tools/train_timeline.py $OUT/tt_$lib > $OUT/train_timeline_$lib.txt 2>&1 || true
  find $OUT/tt_$lib -name '*kernel_trace.csv' -delete
done
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
