set -e
OUT=gpurun_out/r3v; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for f in 0 16 32 64; do
    DG_SH_CU_FREE=$f timeout -k 10 200 python tools/trainer_bench.py --bench-native --steps 200 > $OUT/f$f.$i.log 2>&1
  done
done
DG_SH_CU_FREE=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kp32 -o run -- python3 tools/trainer_bench.py --bench-native --steps 40 > $OUT/kp32.log 2>&1
