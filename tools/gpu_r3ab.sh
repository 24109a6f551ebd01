set -e
OUT=gpurun_out/r3ab; mkdir -p $OUT
export TMPDIR=/tmp
DOGS_HIP_LIB=$(pwd)/ab/fork1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread -k "bitwise or native or overlap" > $OUT/gpu_tests_fork1.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests_fork1.log; exit 0; }
for i in 1 2 3; do
  for v in fork0 fork1; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 200 python tools/trainer_bench.py --bench-native --steps 200 > $OUT/$v.$i.log 2>&1
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 200 python tools/trainer_bench.py --steps 200 > $OUT/admm_$v.$i.log 2>&1
  done
done
