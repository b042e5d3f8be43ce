#!/bin/bash
# round 5 call Q: k_pyr_stream: quad decode hoisted out of the round loop --
# the full -m gpu suite, then per-kernel times against HEAD's build (build/variants/ps_head.so)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_u
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash scripts/variant_kstats.sh r05_u/c3 ps_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_u/c4 ps_head -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_u/c3b ps_head -- --batch 512 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c3b/kstats.txt
