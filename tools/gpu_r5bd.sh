#!/bin/bash
# PMC passes of the final tree's bench workload (tools/profile.sh); pmc_traffic.py / pmc_summary.py run afterwards
OUT=${1:-gpurun_out/r5bd}
bash tools/profile.sh "$OUT/prof" pmc
