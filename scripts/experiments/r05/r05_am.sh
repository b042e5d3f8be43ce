#!/bin/bash
# round 5 call AM: k_match_init phase 2 reads the next batch's list entries one batch ahead --
# -m gpu suite, SearchForInitialization per-call breakdown for the tree and HEAD
# (build/variants/cur_head.so), per-kernel A/B at c3
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_am
mkdir -p $OUT build/headlib
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
cp build/variants/cur_head.so build/headlib/liborb_hip.so && cp orbslam_jpminipc_amd/libsynth.so build/headlib/
hipcc --offload-arch=gfx950 -O2 -w -o build/sfi_breakdown scripts/sfi_breakdown.cpp -Lorbslam_jpminipc_amd -lorb_hip -lsynth -Wl,-rpath,'$ORIGIN/../orbslam_jpminipc_amd' || exit 1
hipcc --offload-arch=gfx950 -O2 -w -o build/sfi_breakdown_head scripts/sfi_breakdown.cpp -Lbuild/headlib -lorb_hip -lsynth -Wl,-rpath,'$ORIGIN/headlib' || exit 1
for rep in 1 2; do
  timeout -k 10 120 ./build/sfi_breakdown > $OUT/bd_new_$rep.json || exit 1
  timeout -k 10 120 ./build/sfi_breakdown_head > $OUT/bd_head_$rep.json || exit 1
done
ldd build/sfi_breakdown_head | grep orb_hip
bash scripts/variant_kstats.sh r05_am/c3 cur_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_am/c3b cur_head -- --batch 512 || exit 1
cat $OUT/bd_*.json $OUT/c3/kstats.txt $OUT/c3b/kstats.txt
