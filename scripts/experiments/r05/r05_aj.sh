#!/bin/bash
# round 5 call AF: k_match_init phase 3 from LDS angles and positions -- -m gpu suite,
# c3 bench step against HEAD (build/variants/cur_head.so) via ORB_HIP_LIB
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_aj
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
  timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err || { echo "bench rc=$?"; tail $OUT/bench_new_$rep.err; exit 1; }
  ORB_HIP_LIB=$PWD/build/variants/cur_head.so timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_head_$rep.json 2> $OUT/bench_head_$rep.err || { echo "bench head rc=$?"; tail $OUT/bench_head_$rep.err; exit 1; }
done
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4))"; done
