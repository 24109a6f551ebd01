set -e
OUT=gpurun_out/r3m; mkdir -p $OUT/ts
export TMPDIR=/tmp
timeout -k 10 60 tools/bin/prio_range > $OUT/prio.txt 2>&1
for i in 1 2; do
  DOGS_HIP_LIB=ab/n9.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/n9.$i.log 2>&1
  DOGS_HIP_LIB=ab/n12.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/n12.$i.log 2>&1
  DG_SH_PRIO=0 DOGS_HIP_LIB=ab/n12.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-admm --no-reference-k > $OUT/ts/n12_p0.$i.log 2>&1
done
DOGS_HIP_LIB=ab/n12.so ROUTES=folded TB_ARGS=--bench-native bash tools/train_timeline.sh $OUT/tt
python3 tools/train_timeline.py $OUT/tt > $OUT/train_timeline.txt 2>&1 || true
find $OUT/tt -name '*kernel_trace.csv' -delete
