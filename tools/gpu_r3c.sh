set -e
OUT=gpurun_out/r3c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py -v -rA --timeout 300 --timeout-method thread > $OUT/trainer_tests.log 2>&1 || echo "trainer tests rc=$?" >> $OUT/trainer_tests.log
bash tools/abn.sh $OUT/ab 2 ab/base.so ab/new.so ab/nosort.so ab/nocomp.so ab/nosortcomp.so
bash tools/profile.sh $OUT/prof
python3 tools/view_timeline.py $OUT/prof/trace/run_kernel_trace.csv > $OUT/view_timeline.txt 2>&1 || true
cp $OUT/prof/trace/*kernel_stats.csv $OUT/ 2>/dev/null || true
rm -f $OUT/prof/trace/*kernel_trace.csv
