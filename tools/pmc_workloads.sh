#!/bin/bash
# PMC passes (tools/profile.sh) of the headline, 4K and sparse 1080p workloads -> profiles/pmc_traffic.json keyed by
# workload (tools/pmc_traffic.py) and per-kernel summaries; raw counter dumps removed (gpurun copy-back limit)
set -e
O=${1:-gpurun_out/pmc6}
mkdir -p $O
export TMPDIR=/tmp
bash tools/profile.sh $O/hd pmc
python3 tools/pmc_traffic.py $O/hd 1000000 1920 1080 > $O/hd_traffic.log 2>&1
python3 tools/pmc_summary.py $O/hd > $O/hd_summary.txt 2>&1
rm -rf $O/hd/pmc* $O/hd/trace/*kernel_trace.csv
BENCH_ARGS="--width 3840 --height 2160" bash tools/profile.sh $O/4k pmc
python3 tools/pmc_traffic.py $O/4k 1000000 3840 2160 > $O/4k_traffic.log 2>&1
python3 tools/pmc_summary.py $O/4k > $O/4k_summary.txt 2>&1
rm -rf $O/4k/pmc* $O/4k/trace/*kernel_trace.csv
BENCH_ARGS="--opacity-mean -2" bash tools/profile.sh $O/sp pmc
python3 tools/pmc_traffic.py $O/sp 1000000 1920 1080 -sparse > $O/sp_traffic.log 2>&1
python3 tools/pmc_summary.py $O/sp > $O/sp_summary.txt 2>&1
rm -rf $O/sp/pmc* $O/sp/trace/*kernel_trace.csv
cp profiles/pmc_traffic.json $O/pmc_traffic.json
