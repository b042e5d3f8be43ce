#!/bin/bash
# Quick GPU iteration: selected tests, then bench (+ optional rocprof) for one workload.
# Usage (via gpurun): bash scripts/gpu_quick.sh TAG "TESTS" [bench args...]
set -o pipefail
TAG=${1:-quick}; TESTS=${2:-tests}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-frames 0 --latency 0 "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step']);print({k:round(v['ms_per_launch'],4) for k,v in d['stages'].items()})"
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --cpu-frames 0 --latency 0 "$@" > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
