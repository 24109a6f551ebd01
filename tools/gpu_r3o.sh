set -e
OUT=gpurun_out/r3o; mkdir -p $OUT/ts
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_trainer.py tests/test_gpu_raster.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
for i in 1 2; do for lib in n9 n14; do
  DOGS_HIP_LIB=ab/$lib.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/$lib.$i.log 2>&1
done; done
DOGS_HIP_LIB=ab/n14.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
