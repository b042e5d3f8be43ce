#!/bin/bash
# round 5 call J: vocabulary + matcher parity after the DPP reductions; BoW leg; per-call latency
set -o pipefail
mkdir -p gpurun_out/r05_j
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vocabulary.py tests/test_gpu_vocabulary_orbvoc.py tests/test_gpu_matcher_family.py tests/test_gpu_bow_batch.py > gpurun_out/r05_j/tests.txt 2>&1 || { tail -40 gpurun_out/r05_j/tests.txt; exit 1; }
tail -1 gpurun_out/r05_j/tests.txt
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 --latency 0 --host-fed 0 > gpurun_out/r05_j/bench_c3.json 2> gpurun_out/r05_j/bench_c3.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05_j/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05_j/bench_c3.json'));print(d['value'],d['ms_per_step']);b=d['bow'];print(b['transform_ms'],b['match_ms'],b['matches_per_pair'])"
