set -e
OUT=gpurun_out/r3p; mkdir -p $OUT/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_admm.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/n14.so ab/n15.so ab/n15_nd.so
