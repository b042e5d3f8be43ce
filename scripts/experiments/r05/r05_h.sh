#!/bin/bash
# round 5 call H: k_pyr_stream per-level task balance (PS_TIMING build) at c3 and c4
set -o pipefail
timeout -k 10 120 python scripts/ps_timing.py build/variants/ps_t.so --batch 512 || exit 1
timeout -k 10 120 python scripts/ps_timing.py build/variants/ps_t.so --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
