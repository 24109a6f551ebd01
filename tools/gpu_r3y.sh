set -e
OUT=gpurun_out/r3y; mkdir -p $OUT/ab
export TMPDIR=/tmp
for v in w8 w16; do
  DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_$v.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests_$v.log; exit 0; }
done
bash tools/abn.sh $OUT/ab 3 ab/w4.so ab/w8.so ab/w16.so
bash tools/kprof.sh $OUT/kp ab/w8.so ab/w16.so
