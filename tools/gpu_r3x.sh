set -e
OUT=gpurun_out/r3x; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for c in 0 288 352 416 512; do
    DOGS_PREFIX_PER_TILE=$c timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train-step --no-admm --no-reference-k > $OUT/c$c.$i.log 2>&1
  done
done
