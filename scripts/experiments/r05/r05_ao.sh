#!/bin/bash
# round 5 call AO: the final session on the committed tree (tests, smoke, c3 bench, rocprof) and
# the c3 PMC passes
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05_v7 || exit 1
bash scripts/pmc_pass.sh r05_v7/pmc_c3 || exit 1
echo done
