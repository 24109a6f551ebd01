set -e
OUT=gpurun_out/r3ah; mkdir -p $OUT
export TMPDIR=/tmp
DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-train-step > $OUT/bench2.json 2> $OUT/bench2.err
