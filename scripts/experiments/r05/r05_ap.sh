#!/bin/bash
# round 5 call AP: k_pyr_stream's rows in pairs with alternating source register sets (no
# register copies between rows) -- pyramid tests, per-kernel A/B at c3 / c4 against HEAD
# (build/variants/cur_head.so), -m gpu, c3 bench step A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_ap
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -k "pyr or pyramid or extract" --timeout 180 --timeout-method thread > $OUT/tests_pyr.txt 2>&1 || { echo "pyr tests rc=$?"; tail -40 $OUT/tests_pyr.txt; exit 1; }
tail -1 $OUT/tests_pyr.txt
bash scripts/variant_kstats.sh r05_ap/c3 cur_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_ap/c4 cur_head -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh r05_ap/c3b cur_head -- --batch 512 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c3b/kstats.txt
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
  timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err || { echo "bench rc=$?"; tail $OUT/bench_new_$rep.err; exit 1; }
  ORB_HIP_LIB=$PWD/build/variants/cur_head.so timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_head_$rep.json 2> $OUT/bench_head_$rep.err || { echo "bench head rc=$?"; tail $OUT/bench_head_$rep.err; exit 1; }
done
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4))"; done
