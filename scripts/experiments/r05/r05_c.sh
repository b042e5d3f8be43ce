#!/bin/bash
# round 5 call C: probe of the pattern registers, corner-list fallback parity, bench with the BoW leg
set -o pipefail
mkdir -p gpurun_out/r05_c
REPS=10 ./scripts/r05_diag.sh odt_probe || exit 1
grep -c "probe:" gpurun_out/r05_diag/odt_probe.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fast_fallback.py > gpurun_out/r05_c/tests.txt 2>&1 || { tail -40 gpurun_out/r05_c/tests.txt; exit 1; }
tail -3 gpurun_out/r05_c/tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 --latency 0 --host-fed 0 > gpurun_out/r05_c/bench_c3.json 2> gpurun_out/r05_c/bench_c3.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05_c/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05_c/bench_c3.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['bow'],indent=1))"
