#!/bin/bash
# round 5 call L: k_fast with the SWAR compass -- parity (extraction tests), then per-kernel
# times against the previous compass (build/variants/kf_old.so) at c3 and c4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fast_fallback.py tests/test_gpu_configs.py tests/test_gpu_pyramid_stream.py > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash scripts/variant_kstats.sh r05_l/c3 kf_old -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_l/c4 kf_old -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_l/c3b kf_old -- --batch 512 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c3b/kstats.txt
