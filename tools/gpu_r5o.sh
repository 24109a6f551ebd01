#!/bin/bash
# sigmoid backward in torch's association + capacity-context isolation test: the first-step probe, then the evidence
# run (whole -m gpu suite, smoke, bench, kernel trace, 2-rank gloo rehearsal)
OUT=${1:-gpurun_out/r5o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/first_step_probe.py > "$OUT/first_step.log" 2>&1 || exit $?
bash tools/gpu_r5i.sh "$OUT"
