#!/bin/bash
# round 5 call O: the full session on the current tree (tests, smoke, c3 bench, rocprof), then
# c4 bench + rocprof and the PMC passes for c3 / c4 (k_orient_desc changed)
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_round.sh r05_v2 || exit 1
OUT=gpurun_out/r05_v2
timeout -k 10 600 python bench.py --workload c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python bench.py --workload c4 --cpu-frames 0 --latency 0 --host-fed 0 > $OUT/prof_c4.log 2>&1 || { echo "rocprof c4 rc=$?"; exit 1; }
bash scripts/pmc_pass.sh r05_v2/pmc_c3 || exit 1
bash scripts/pmc_pass.sh r05_v2/pmc_c4 --workload c4 || exit 1
echo done
