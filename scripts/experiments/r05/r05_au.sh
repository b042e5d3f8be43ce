#!/bin/bash
# round 5 call AU: smoke, the k_orient_desc determinism screen and the c3 bench on the final tree
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_v9
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
REPS=6 bash scripts/r05_diag.sh intree || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'], 4))"
