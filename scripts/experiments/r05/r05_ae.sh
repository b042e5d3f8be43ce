#!/bin/bash
# round 5 call AD: k_rerun with the eight-point pre-test --
# -m gpu suite, then per-kernel times against HEAD (build/variants/kr_c4pt.so) at c3 / c4 / c5
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_ae
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash scripts/variant_kstats.sh r05_ae/c3 kr_c4pt -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_ae/c4 kr_c4pt -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_ae/c5 kr_c4pt -- --batch 512 --width 1280 --height 720 --nfeatures 2500 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c5/kstats.txt
