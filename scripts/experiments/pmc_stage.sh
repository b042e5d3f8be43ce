#!/bin/bash
# SQ instruction-mix PMC pass over stage_times.py (one library build).  Usage: pmc_stage.sh TAG [LIB]
TAG=$1; LIB=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $OUT/sq -o run --output-format csv -- python scripts/stage_times.py $LIB --batch 512 --steps 2 > $OUT/sq.log 2>&1
