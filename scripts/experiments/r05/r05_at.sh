#!/bin/bash
# round 5 call AT: k_pyr_resize (per-level pyramid: batches < 256, single frames, colour) with
# k_pyr_stream's paired rows -- pyramid / extraction tests, per-kernel A/B at B = 128 against HEAD
# (build/variants/cur_head.so), -m gpu
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_at
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -k "pyr or pyramid or extract or colour or color" --timeout 180 --timeout-method thread > $OUT/tests_pyr.txt 2>&1 || { echo "pyr tests rc=$?"; tail -40 $OUT/tests_pyr.txt; exit 1; }
tail -1 $OUT/tests_pyr.txt
bash scripts/variant_kstats.sh r05_at/c3b128 cur_head -- --batch 128 || exit 1
bash scripts/variant_kstats.sh r05_at/c3b128b cur_head -- --batch 128 || exit 1
cat $OUT/c3b128/kstats.txt $OUT/c3b128b/kstats.txt
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
