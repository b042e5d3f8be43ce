#!/bin/bash
# round 5 call D: trig-on-wave-3 screen, batched BoW parity (16 waves) and the BoW bench leg
set -o pipefail
mkdir -p gpurun_out/r05_d
REPS=10 ./scripts/r05_diag.sh odt_trig3 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bow_batch.py > gpurun_out/r05_d/tests.txt 2>&1 || { tail -40 gpurun_out/r05_d/tests.txt; exit 1; }
tail -2 gpurun_out/r05_d/tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 --latency 0 --host-fed 0 > gpurun_out/r05_d/bench_c3.json 2> gpurun_out/r05_d/bench_c3.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05_d/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05_d/bench_c3.json'));print(d['value'],d['ms_per_step']);b=d['bow'];print(b['transform_ms'],b['match_ms'],b['matches_per_pair'])"
bash scripts/variant_kstats.sh r05_d/c3 od_preblur -- --batch 512 || exit 1
bash scripts/variant_kstats.sh r05_d/c4 od_preblur -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
cat gpurun_out/r05_d/c3/kstats.txt gpurun_out/r05_d/c4/kstats.txt
