#!/bin/bash
# round 5 call I: SFI phase timing after the phase-1 load change; parity; c3 kernel stats
set -o pipefail
mkdir -p gpurun_out/r05_i
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sfi_stress.py > gpurun_out/r05_i/tests.txt 2>&1 || { tail -30 gpurun_out/r05_i/tests.txt; exit 1; }
tail -1 gpurun_out/r05_i/tests.txt
timeout -k 10 120 python scripts/km_timing.py build/variants/km_t.so --per 2 | tail -1 || exit 1
timeout -k 10 120 python scripts/km_timing.py build/variants/km_t.so --per 512 | tail -1 || exit 1
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 || exit 1
bash scripts/variant_kstats.sh r05_i/c3 -- --batch 512 || exit 1
cat gpurun_out/r05_i/c3/kstats.txt
