#!/bin/bash
# Bench one workload at several batch shapes (no CPU leg / latency), stage times per run.
# Usage (via gpurun): bash scripts/bench_sweep.sh TAG WORKLOAD "ARGS1" "ARGS2" ...
set -o pipefail
TAG=$1; WL=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for a in "$@"; do
  timeout -k 10 300 python bench.py --workload $WL --cpu-frames 0 --latency 0 $a > $OUT/sweep_$i.json 2> $OUT/sweep_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench '$a' rc=$rc"; tail -5 $OUT/sweep_$i.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/sweep_$i.json'));c=d['config'];print('$WL', '$a', 'B=%d'%c['batch_per_gpu'], round(d['value']), round(d['ms_per_step'],3), {k:round(v['ms_per_launch'],4) for k,v in d['stages'].items()})" | tee -a $OUT/sweep.txt
  i=$((i+1))
done
