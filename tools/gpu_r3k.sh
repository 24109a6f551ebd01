set -e
OUT=gpurun_out/r3k; mkdir -p $OUT/ab $OUT/ts
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
for i in 1 2 3; do for lib in n9 n10; do
  DOGS_HIP_LIB=ab/$lib.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/$lib.$i.log 2>&1
done; done
DOGS_HIP_LIB=ab/n10.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
