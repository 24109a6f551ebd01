#!/bin/bash
set -e
export TMPDIR=/tmp
B="bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-train-step --no-reference-k --no-admm --no-sweep"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pl1 -o run -- python3 $B > gpurun_out/pl1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACCUM_PREV_HIRES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/pl2 -o run -- python3 $B > gpurun_out/pl2.log 2>&1
