#!/bin/bash
# round 5 call K: c4 / c5 benches with rocprof kernel stats, PMC passes for c3 / c4 / c5
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_k
mkdir -p $OUT
for w in c4 c5; do
  timeout -k 10 600 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w rc=$?"; tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));print('$w', d['value'], d['ms_per_step'])"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run --output-format csv -- python bench.py --workload $w --cpu-frames 0 --latency 0 --host-fed 0 > $OUT/prof_$w.log 2>&1 || { echo "rocprof $w rc=$?"; exit 1; }
done
bash scripts/pmc_pass.sh r05_k/pmc_c3 || exit 1
bash scripts/pmc_pass.sh r05_k/pmc_c4 --workload c4 || exit 1
bash scripts/pmc_pass.sh r05_k/pmc_c5 --workload c5 || exit 1
echo done
