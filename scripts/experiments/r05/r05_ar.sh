#!/bin/bash
# round 5 call AR: the final session on the committed tree (tests, smoke, c3 bench, rocprof), the
# c3 PMC passes, and the k_orient_desc determinism screen (scripts/r05_diag.sh) on the in-tree
# library
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05_v8 || exit 1
bash scripts/pmc_pass.sh r05_v8/pmc_c3 || exit 1
REPS=6 bash scripts/r05_diag.sh intree || exit 1
echo done
