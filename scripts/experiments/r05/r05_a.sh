#!/bin/bash
# round 5 call A: k_orient_desc diagnosis variants, stream-hook tests, replicas test, short bench
set -o pipefail
mkdir -p gpurun_out/r05_a
REPS=10 ./scripts/r05_diag.sh odt odt_asmwait odt_sc odt_dw odt_malloc intree || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_replicas.py > gpurun_out/r05_a/tests.txt 2>&1 || { tail -30 gpurun_out/r05_a/tests.txt; exit 1; }
tail -3 gpurun_out/r05_a/tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 > gpurun_out/r05_a/bench_c3.json 2> gpurun_out/r05_a/bench_c3.err || { tail -20 gpurun_out/r05_a/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05_a/bench_c3.json'));print(d['value'],d['ms_per_step'],d['host_fed']['value'],d['host_fed']['ms_per_step'],d['config']['gpu_max_hw_queues'],d['latency_b1'])"
