set -e
OUT=gpurun_out/r3l; mkdir -p $OUT/ts
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> $OUT/gpu_tests.log; exit 0; }
for i in 1 2; do
  DOGS_HIP_LIB=ab/n9.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/n9.$i.log 2>&1
  for nb in 256 512 1024; do
    DG_SH_ADAM_BLOCKS=$nb DOGS_HIP_LIB=ab/n11.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/n11_$nb.$i.log 2>&1
  done
done
for nb in 256 512; do
  DG_SH_ADAM_BLOCKS=$nb DOGS_HIP_LIB=ab/n11.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt_$nb
  python3 tools/train_timeline.py $OUT/tt_$nb > $OUT/train_timeline_$nb.txt 2>&1 || true
  find $OUT/tt_$nb -name '*kernel_trace.csv' -delete
done
