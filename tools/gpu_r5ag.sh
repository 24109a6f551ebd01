mkdir -p gpurun_out/r5ag
B="--steps 4 --warmup 1 --no-sweep --no-admm --no-train-step --no-cpu-baseline --no-reference-k"
DOGS_HIP_LIB=ab/bstats.so timeout -k 10 200 python bench.py $B > gpurun_out/r5ag/1e6.log 2>&1 && \
DOGS_HIP_LIB=ab/bstats.so timeout -k 10 200 python bench.py $B --gaussians 100000 > gpurun_out/r5ag/1e5.log 2>&1
