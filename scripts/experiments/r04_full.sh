#!/bin/bash
# Full round-4 GPU session: gpu_round.sh (tests, smoke, bench, rocprof) plus the k_rerun phase
# split and the available-counter list.
set -o pipefail
TAG=${1:-r04_full}
bash scripts/gpu_round.sh $TAG || exit $?
OUT=gpurun_out/$TAG
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
if [ -f build/variants/krtiming.so ]; then
  timeout -k 10 120 python scripts/kr_timing.py build/variants/krtiming.so 1241 376 2000 512 > $OUT/kr_c4.txt 2>&1 || exit 1
  timeout -k 10 180 python scripts/kr_timing.py build/variants/krtiming.so 1280 720 2500 512 > $OUT/kr_c5.txt 2>&1 || exit 1
  cat $OUT/kr_c4.txt $OUT/kr_c5.txt
fi
cat $OUT/summary.txt
