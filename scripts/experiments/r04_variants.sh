#!/bin/bash
# Parity of build/variants/NAME.so (ORB_HIP_LIB) on the core parity file + the c3 bench batch for
# each NAME given, then rocprofv3 kernel means of the in-tree build and the variants at c3/c4/c5.
# Usage: bash scripts/r04_variants.sh TAG NAME...
set -o pipefail
TAG=${1:-r04_var}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  ORB_HIP_LIB=build/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_bench_batch_full_parity" -x -q --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed rc=$?"; tail -30 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
bash scripts/variant_kstats.sh $TAG/c3 "$@" -- --batch 512 || exit 1
bash scripts/variant_kstats.sh $TAG/c4 "$@" -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh $TAG/c5 "$@" -- --batch 512 --width 1280 --height 720 --nfeatures 2500 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c5/kstats.txt
