#!/bin/bash
# round 5 call M: k_orient_desc with one IC table and the row-pass fragments through opaque SGPR bases --
# nondeterminism screen (od_diag, 10 repetitions), extraction parity tests, then per-kernel times
# against HEAD's build (build/variants/od_head.so) at c3 and c4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_p
mkdir -p $OUT
REPS=10 bash scripts/r05_diag.sh intree || exit 1
cp gpurun_out/r05_diag/intree.txt $OUT/diag_intree.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py tests/test_gpu_facade.py > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash scripts/variant_kstats.sh r05_p/c3 od_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_p/c4 od_head -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_p/c3b od_head -- --batch 512 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c3b/kstats.txt
