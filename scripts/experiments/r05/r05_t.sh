#!/bin/bash
# round 5 call T: k_pyr_stream variants -- both changes (in-tree), the decode not hoisted
# (ps_noh), the border indices hoisted again (ps_nob), HEAD (ps_head)
set -o pipefail
export TMPDIR=/tmp
bash scripts/variant_kstats.sh r05_t/c3 ps_noh ps_nob ps_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_t/c3b ps_noh ps_nob ps_head -- --batch 512 || exit 1
cat gpurun_out/r05_t/c3/kstats.txt gpurun_out/r05_t/c3b/kstats.txt
