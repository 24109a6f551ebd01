set -e
OUT=gpurun_out/r3ac; mkdir -p $OUT/ab
export TMPDIR=/tmp
DOGS_HIP_LIB=$(pwd)/ab/pad30.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_pad30.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests_pad30.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/pad0.so ab/pad30.so ab/pad14.so
bash tools/kprof.sh $OUT/kp ab/pad30.so
