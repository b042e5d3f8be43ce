#!/bin/bash
# host-fed schedule experiments (scripts/hostfed_modes.py)
set -o pipefail
OUT=gpurun_out/${1:-r04_hf}
mkdir -p $OUT
timeout -k 10 300 python scripts/hostfed_modes.py > $OUT/modes.txt 2>&1 || { echo "modes failed rc=$?"; tail $OUT/modes.txt; exit 1; }
cat $OUT/modes.txt
