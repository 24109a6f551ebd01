#!/bin/bash
# Instruction-cache counters of the bench workload (one PMC pass).
set -e
export TMPDIR=/tmp
B="bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-train-step --no-reference-k --no-admm"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH_LEVEL SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/pi1 -o run -- python3 $B > gpurun_out/pi1.log 2>&1
