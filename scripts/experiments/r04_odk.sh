#!/bin/bash
# k_orient_desc slots-per-wave A/B: parity (tests/test_gpu_parity.py + the c3 bench batch) of
# each variant given (ORB_HIP_LIB), then the kernel means of base (HEAD) and the variants at
# c3 / c4.  Usage: bash scripts/r04_odk.sh TAG VARIANT...
set -o pipefail
TAG=${1:-r04_odk}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = "base" ] && continue
  ORB_HIP_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_bench_batch_full_parity" -x -q --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed rc=$?"; tail -30 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
bash scripts/variant_kstats.sh $TAG/c3 "$@" -- --batch 512 || exit 1
bash scripts/variant_kstats.sh $TAG/c4 "$@" -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt
