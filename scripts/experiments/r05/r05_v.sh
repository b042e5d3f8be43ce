#!/bin/bash
# round 5 call V: the full session on the current tree (tests, smoke, c3 bench, rocprof), then
# c4 / c5 benches + rocprof and the PMC passes for c3 / c4 / c5
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05_v3 || exit 1
OUT=gpurun_out/r05_v3
for w in c4 c5; do
  timeout -k 10 600 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w rc=$?"; exit 1; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run --output-format csv -- python bench.py --workload $w --cpu-frames 0 --latency 0 --host-fed 0 > $OUT/prof_$w.log 2>&1 || { echo "rocprof $w rc=$?"; exit 1; }
done
bash scripts/pmc_pass.sh r05_v3/pmc_c3 || exit 1
bash scripts/pmc_pass.sh r05_v3/pmc_c4 --workload c4 || exit 1
bash scripts/pmc_pass.sh r05_v3/pmc_c5 --workload c5 || exit 1
echo done
