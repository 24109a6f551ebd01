set -e
OUT=gpurun_out/r3ak; mkdir -p $OUT/ab
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_aux.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/wb0.so ab/wb1.so
