#!/bin/bash
# round 5 call AC: k_rerun without its cell staging (timing-only ablation, wrong output) at c4/c5
set -o pipefail
export TMPDIR=/tmp
bash scripts/variant_kstats.sh r05_ac/c4 kr_nostage -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_ac/c5 kr_nostage -- --batch 512 --width 1280 --height 720 --nfeatures 2500 || exit 1
cat gpurun_out/r05_ac/c4/kstats.txt gpurun_out/r05_ac/c5/kstats.txt
