set -e
OUT=gpurun_out/r3al; mkdir -p $OUT/ab
export TMPDIR=/tmp
DOGS_HIP_LIB=$(pwd)/ab/ff1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_ff1.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests_ff1.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/ff0.so ab/ff1.so
