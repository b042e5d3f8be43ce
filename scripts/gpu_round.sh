#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash scripts/gpu_round.sh TAG [bench args...]
# Any abnormal end of a GPU step (fault, abort, segfault, time limit: rc not 0/1) ends the
# session there; an ordinary test failure (rc 1) still lets the bench run.
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step NAME RC
    echo "$1 rc=$2" | tee -a $OUT/summary.txt
    if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "abnormal end of $1: stopping" | tee -a $OUT/summary.txt; exit "$2"; fi
}
timeout -k 10 900 python -u -m pytest tests -q -m gpu --maxfail=5 --timeout 180 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log >> $OUT/summary.txt; step pytest_gpu $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1
step smoke $?
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
step bench $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-frames 0 --latency 0 --host-fed 0 "$@" > $OUT/prof.log 2>&1
step rocprof $?
