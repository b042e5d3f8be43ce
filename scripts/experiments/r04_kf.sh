#!/bin/bash
# k_fast variant A/B: parity of each variant (ORB_HIP_LIB: core parity file + the c3 and c4
# bench batches), kernel means at c3 / c4 / c5 (B = 4096), and the per-phase probes of the
# k_fast timing builds present (kftiming.so, kftpair.so).  Usage: bash scripts/r04_kf.sh TAG VARIANT...
set -o pipefail
TAG=${1:-r04_kf}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = "base" ] && continue
  ORB_HIP_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_bench_batch_full_parity" "tests/test_gpu_configs.py::test_bench_batch_c4_full_parity" -x -q --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed rc=$?"; tail -30 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
bash scripts/variant_kstats.sh $TAG/c3 "$@" -- --batch 512 || exit 1
bash scripts/variant_kstats.sh $TAG/c4 "$@" -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh $TAG/c5 "$@" -- --batch 4096 --width 1280 --height 720 --nfeatures 2500 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c5/kstats.txt
for v in kftiming kftpair; do
  [ -f build/variants/$v.so ] || continue
  timeout -k 10 120 python scripts/kf_timing.py build/variants/$v.so > $OUT/kf_$v.txt 2>&1 || exit 1
  echo "== $v"; tail -2 $OUT/kf_$v.txt
done
