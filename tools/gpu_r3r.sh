set -e
OUT=gpurun_out/r3r; mkdir -p $OUT/ab
export TMPDIR=/tmp DOGS_TEST_LOG=$OUT/fullsize.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py tests/test_gpu_admm.py tests/test_gpu_aux.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
bash tools/abn.sh $OUT/ab 3 ab/n16.so ab/n17.so ab/n17_pp1.so ab/n17_pp4.so ab/lc32.so ab/lc64.so
