#!/bin/bash
# k_pyr_stream experiments: phase timing of PS_TIMING variants + stage times of variants.
# Usage (via gpurun): bash scripts/ps_exp.sh TAG "TIMING_VARIANTS" "STAGE_VARIANTS"
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in $2; do
  for wl in "--width 640 --height 480 --nfeatures 1000" "--width 1280 --height 720 --nfeatures 2500"; do
    echo "== $v $wl" >> $OUT/pst.txt
    timeout -k 10 120 python scripts/ps_timing.py build/variants/$v.so $wl >> $OUT/pst.txt 2>&1 || exit $?
  done
done
timeout -k 10 120 python scripts/stage_times.py --batch 512 >> $OUT/times.txt 2>>$OUT/err.txt || exit $?
for v in $3; do
  timeout -k 10 120 python scripts/stage_times.py build/variants/$v.so --batch 512 >> $OUT/times.txt 2>>$OUT/err.txt || exit $?
done
grep -v amdgpu.ids $OUT/pst.txt; cat $OUT/times.txt
