set -e
OUT=gpurun_out/r3ai; mkdir -p $OUT/ab
export TMPDIR=/tmp
DOGS_HIP_LIB=$(pwd)/ab/lc32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_lc32.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests_lc32.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/k0.so ab/s1.so ab/s4.so ab/lc8.so ab/lc32.so
