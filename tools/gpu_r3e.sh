set -e
OUT=gpurun_out/r3e; mkdir -p $OUT
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/new3.so ab/new3_2l.so
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
