#!/bin/bash
# PMC passes (each in its own rocprofv3 run, kernel-trace only) over bench.py.
# Usage: bash scripts/pmc_pass.sh TAG [bench args...]
# Pass 1/2 give the HBM-side bytes (FETCH_SIZE / WRITE_SIZE, one TCC group each); pass 3 the
# SQ instruction mix.  Summarise with scripts/pmc_summary.py gpurun_out/TAG.
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o run --output-format csv -- python bench.py --cpu-frames 0 --latency 0 --host-fed 0 --steps 5 --warmup 1 --survey-steps 1 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
