#!/bin/bash
# the bench step serial vs the two stream-overlap schedules (--overlap 1 / 2) at c3 and c4
set -o pipefail
OUT=gpurun_out/${1:-r04_ov}
mkdir -p $OUT
for wl in c3 c4; do
  for ov in 0 1 2 0; do
    timeout -k 10 200 python bench.py --workload $wl --overlap $ov --cpu-frames 0 --latency 0 --host-fed 0 --steps 30 > $OUT/b_${wl}_$ov.json 2> $OUT/b_${wl}_$ov.err || { echo "bench $wl $ov failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${wl}_$ov.json'));print('$wl overlap $ov', round(d['value']), round(d['ms_per_step'],4))"
  done
done
