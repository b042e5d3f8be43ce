#!/bin/bash
# round 5 call AV: long k_orient_desc determinism screen on the final tree (40 repetitions x 3
# frames x 2000 keypoints at 640x480)
set -o pipefail
export TMPDIR=/tmp
REPS=40 bash scripts/r05_diag.sh intree || exit 1
echo done
