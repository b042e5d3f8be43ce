#!/bin/bash
# round 5 call W: k_match_init with 16-wave workgroups below 256 pairs; SFI host call with the
# kernel reading / writing the pinned staging (ORB_SFI_ZERO_COPY=1) -- -m gpu suite with and
# without zero copy, then the per-call breakdown both ways
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_w
mkdir -p $OUT build
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
ORB_SFI_ZERO_COPY=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -k "match or sfi or init or facade" > $OUT/tests_zc.txt 2>&1 || { echo "zc tests rc=$?"; tail -30 $OUT/tests_zc.txt; exit 1; }
tail -1 $OUT/tests_zc.txt
hipcc --offload-arch=gfx950 -O2 -w -o build/sfi_breakdown scripts/sfi_breakdown.cpp -Lorbslam_jpminipc_amd -lorb_hip -lsynth -Wl,-rpath,'$ORIGIN/../orbslam_jpminipc_amd' || exit 1
timeout -k 10 120 ./build/sfi_breakdown > $OUT/bd_copy.json && ORB_SFI_ZERO_COPY=1 timeout -k 10 120 ./build/sfi_breakdown > $OUT/bd_zc.json || exit 1
cat $OUT/bd_copy.json $OUT/bd_zc.json
