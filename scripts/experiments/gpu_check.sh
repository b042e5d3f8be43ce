#!/bin/bash
# Quick GPU session: parity tests, bench, per-stage times of the in-tree build and of the
# ablation variants in build/variants (scripts/build_variant.sh).
# Usage (via gpurun): bash scripts/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {
    echo "$1 rc=$2" | tee -a $OUT/summary.txt
    if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then echo "abnormal end of $1: stopping" | tee -a $OUT/summary.txt; exit "$2"; fi
}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log >> $OUT/summary.txt; step pytest_gpu $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
step bench $?
for lib in "" build/variants/*.so; do
  timeout -k 10 120 python scripts/stage_times.py $lib >> $OUT/stages.jsonl 2>> $OUT/stages.err
  step "stages $lib" $?
done
