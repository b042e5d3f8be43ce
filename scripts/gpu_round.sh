#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash scripts/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1
echo "pytest_gpu rc=$?" | tee -a $OUT/summary.txt
tail -3 $OUT/pytest_gpu.log >> $OUT/summary.txt
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1
echo "smoke rc=$?" | tee -a $OUT/summary.txt
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?" | tee -a $OUT/summary.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-frames 0 "$@" > $OUT/prof.log 2>&1
echo "rocprof rc=$?" | tee -a $OUT/summary.txt
