#!/bin/bash
# PMC passes (each in its own rocprofv3 run, kernel-trace only) for the extraction kernels.
# Usage: bash scripts/pmc_pass.sh TAG [bench args...]
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python bench.py --cpu-frames 0 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
