#!/bin/bash
OUT=${1:-gpurun_out/r5g}
mkdir -p "$OUT"
export TMPDIR=/tmp
MIOPEN_FIND_MODE=FAST timeout -k 10 400 python -u tools/mask_conc_probe.py > "$OUT/mask_conc_fast.log" 2>&1
MIOPEN_DEBUG_DISABLE_FIND_DB=1 MIOPEN_DISABLE_CACHE=1 timeout -k 10 400 python -u tools/mask_conc_probe.py > "$OUT/mask_conc_nodb.log" 2>&1
