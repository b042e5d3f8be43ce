#!/bin/bash
# round 5 call B: exit-with-outstanding-load screens, batched BoW + stream tests, bench exit code
set -o pipefail
mkdir -p gpurun_out/r05_b
REPS=10 ./scripts/r05_diag.sh odt_drainexit odt_prewait ship_exitload || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bow_batch.py tests/test_gpu_streams.py > gpurun_out/r05_b/tests.txt 2>&1 || { tail -40 gpurun_out/r05_b/tests.txt; exit 1; }
tail -3 gpurun_out/r05_b/tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 --latency 0 > gpurun_out/r05_b/bench_c3.json 2> gpurun_out/r05_b/bench_c3.err; echo "bench rc=$?"
python -c "import json;d=json.load(open('gpurun_out/r05_b/bench_c3.json'));print(d['value'],d['ms_per_step'],d['host_fed']['value'])"
