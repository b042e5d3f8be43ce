#!/bin/bash
# Bench + rocprofv3 kernel stats (+ PMC passes with PMC=1) for every BASELINE workload preset.
# Usage (via gpurun): bash scripts/bench_all.sh TAG [workloads...]   (default: c3 c4 c5)
set -o pipefail
TAG=${1:-all}; shift
WLS=${@:-c3 c4 c5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for wl in $WLS; do
  timeout -k 10 400 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err
  rc=$?; echo "bench $wl rc=$rc" | tee -a $OUT/summary.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$wl -o run --output-format csv -- python bench.py --workload $wl --cpu-frames 0 --latency 0 --host-fed 0 > $OUT/prof_$wl.log 2>&1
  rc=$?; echo "rocprof $wl rc=$rc" | tee -a $OUT/summary.txt; [ $rc -eq 0 ] || exit $rc
  if [ "${PMC:-0}" = "1" ]; then
    bash scripts/pmc_pass.sh $TAG/pmc_$wl --workload $wl >> $OUT/summary.txt 2>&1
    rc=$?; echo "pmc $wl rc=$rc" | tee -a $OUT/summary.txt; [ $rc -eq 0 ] || exit $rc
  fi
done
