#!/bin/bash
# round 5 call E: run-to-run screens (GPU vs GPU) of trig-wave ablations of the pointer-table variant
set -o pipefail
ORB_DIAG_SELF=1 REPS=10 ./scripts/r05_diag.sh odt odt_nof64 odt_nodiv odt_notrig || exit 1
