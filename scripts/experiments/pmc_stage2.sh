#!/bin/bash
# SQ wave-state PMC pass over stage_times.py.  Usage: pmc_stage2.sh TAG [LIB]
TAG=$1; LIB=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES -d $OUT/sq2 -o run --output-format csv -- python scripts/stage_times.py $LIB --batch 512 --steps 2 > $OUT/sq2.log 2>&1
