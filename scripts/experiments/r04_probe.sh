#!/bin/bash
# Timing-probe builds only (no parity): k_pyr_stream per-level task time per round.
set -o pipefail
OUT=gpurun_out/${1:-r04_probe}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/ps_timing.py build/variants/pstiming.so > $OUT/ps_c3.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/ps_timing.py build/variants/pstiming.so --width 1241 --height 376 --nfeatures 2000 > $OUT/ps_c4.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/ps_timing.py build/variants/pstiming.so --width 1280 --height 720 --nfeatures 2500 > $OUT/ps_c5.txt 2>&1 || exit 1
cat $OUT/ps_c3.txt $OUT/ps_c4.txt $OUT/ps_c5.txt
