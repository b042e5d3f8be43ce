#!/bin/bash
# round 5 call AQ: k_orient_desc's py * (cos, -sin) with py splat by op_sel (no copy per sample) --
# descriptor tests first, then -m gpu, per-kernel A/B against HEAD
# (build/variants/cur_head.so) at c3 / c4, c3 bench step
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_aq
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x -k "desc or extract or parity" --timeout 180 --timeout-method thread > $OUT/tests_desc.txt 2>&1 || { echo "desc tests rc=$?"; tail -40 $OUT/tests_desc.txt; exit 1; }
tail -1 $OUT/tests_desc.txt
bash scripts/variant_kstats.sh r05_aq/c3 cur_head -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_aq/c4 cur_head -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for rep in 1 2; do
  timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err || { echo "bench rc=$?"; tail $OUT/bench_new_$rep.err; exit 1; }
  ORB_HIP_LIB=$PWD/build/variants/cur_head.so timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 > $OUT/bench_head_$rep.json 2> $OUT/bench_head_$rep.err || { echo "bench head rc=$?"; tail $OUT/bench_head_$rep.err; exit 1; }
done
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],4))"; done
