#!/bin/bash
# Bench the in-tree library and each build/variants/*.so given (GPU box), REPS rounds alternating
# the builds (A B C A B C ...) so box drift hits all alike: value and per-stage ms per run.
# Usage: REPS=3 bash scripts/variant_bench.sh TAG "BENCH ARGS" variant1 variant2 ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-1}); do
for v in intree "$@"; do
  if [ "$v" = intree ]; then L=""; else L=$PWD/build/variants/$v.so; fi
  ORB_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-frames 0 --latency 0 --steps 10 $ARGS > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -3 $OUT/$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', round(d['value']), round(d['ms_per_step'],4), {k:round(x['ms_per_launch'],4) for k,x in d['stages'].items()})" | tee -a $OUT/summary.txt
done
done
