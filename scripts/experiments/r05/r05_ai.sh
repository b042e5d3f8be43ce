#!/bin/bash
# round 5 call AI: the two-stream pipelined step modes (--overlap 1 / 2) against the serial step
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_ai
mkdir -p $OUT
for ov in 0 1 2 0; do
  timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 --latency 0 --bow 0 --steps 50 --overlap $ov > $OUT/bench_ov$ov.json 2> $OUT/bench_ov$ov.err || { echo "bench ov$ov rc=$?"; tail $OUT/bench_ov$ov.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_ov$ov.json').read().strip().splitlines()[-1]); print('overlap $ov', round(d['value']), round(d['ms_per_step'],4))"
done
