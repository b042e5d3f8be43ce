#!/bin/bash
# round 5 call Y: k_fast with four dwords per lane and compass step (kf_dpl4) against HEAD
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 env ORB_HIP_LIB=$PWD/build/variants/kf_dpl4.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fast_fallback.py > gpurun_out/r05_y_tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r05_y_tests.txt; exit 1; }
tail -1 gpurun_out/r05_y_tests.txt
bash scripts/variant_kstats.sh r05_y/c3 kf_dpl4 -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_y/c4 kf_dpl4 -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
cat gpurun_out/r05_y/c3/kstats.txt gpurun_out/r05_y/c4/kstats.txt
