#!/bin/bash
# round 5 call AB: k_bow_pairs with both frames staged in LDS and the rotation histogram built
# after the node loop -- -m gpu suite, the C++ per-call latencies, the c3 bench (bow block)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_ab
mkdir -p $OUT build
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
python -c "import pathlib, subprocess, __graft_entry__ as g; subprocess.check_call(g.LATENCY_CMD(pathlib.Path('build/latency_gpu').resolve()))" || exit 1
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 > $OUT/latency.json || exit 1
timeout -k 10 600 python bench.py --cpu-frames 0 --host-fed 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail $OUT/bench.err; exit 1; }
cat $OUT/latency.json
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); b=d['bow']; print(d['value'], b['transform_ms'], b['match_ms'])"
