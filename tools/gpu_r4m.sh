#!/bin/bash
# Round 4: same-box A/B of the forward's counter publish (k_depth_cut vs the phase-1 render's first block): the raster
# bench and both training routes, interleaved.
set -e
OUT=${1:-gpurun_out/r4m}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/abn.sh "$OUT/ab" 3 ab/hc_render.so ab/hc_cut.so
for r in 1 2; do
  for v in hc_render hc_cut; do
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-autograd --steps 100 \
        > "$OUT/ag_$v.$r.txt" 2>&1
    DOGS_HIP_LIB=$(pwd)/ab/$v.so timeout -k 10 300 python tools/trainer_bench.py --bench-native --steps 100 \
        > "$OUT/nat_$v.$r.txt" 2>&1
  done
done
