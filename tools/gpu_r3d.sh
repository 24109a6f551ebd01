set -e
OUT=gpurun_out/r3d; mkdir -p $OUT
export TMPDIR=/tmp
for v in split fat2 fat14 splitfat; do
  DOGS_HIP_LIB=ab/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_boundary.py "tests/test_gpu_fullsize.py::test_fullsize_views_match_oracle[1e6-1080p]" "tests/test_gpu_fullsize.py::test_fullsize_views_match_oracle[5e6-1080p]" -x -q --timeout 300 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed rc=$?" >> $OUT/parity_$v.log; }
done
bash tools/abn.sh $OUT/ab 3 ab/cur.so ab/split.so ab/fat2.so ab/fat12.so ab/fat14.so ab/fat2x8.so ab/splitfat.so
