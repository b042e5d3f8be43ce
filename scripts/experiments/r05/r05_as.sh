#!/bin/bash
# round 5 call AS: c4 and c5 bench lines on the final tree (default legs)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_v8
mkdir -p $OUT
for w in c4 c5; do
  timeout -k 10 900 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w rc=$?"; tail $OUT/bench_$w.err; exit 1; }
  tail -1 $OUT/bench_$w.json | cut -c1-200
done
echo done
