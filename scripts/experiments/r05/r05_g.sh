#!/bin/bash
# round 5 call G: matcher-family parity after the resolver / BoW per-call changes, then latency
set -o pipefail
mkdir -p gpurun_out/r05_g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_matcher_family.py tests/test_gpu_bow_batch.py tests/test_gpu_facade.py "tests/test_gpu_parity.py::test_search_for_initialization_parity" > gpurun_out/r05_g/tests.txt 2>&1 || { tail -40 gpurun_out/r05_g/tests.txt; exit 1; }
tail -2 gpurun_out/r05_g/tests.txt
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 > gpurun_out/r05_g/lat_c3.json || exit 1
cat gpurun_out/r05_g/lat_c3.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_g/prof -o run --output-format csv -- ./build/latency_gpu 640 480 1000 50 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05_g/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
timeout -k 10 120 python scripts/km_timing.py build/variants/km_t.so --per 2 || exit 1
timeout -k 10 120 python scripts/km_timing.py build/variants/km_t.so --per 512 || exit 1
#!/bin/bash
set -o pipefail
timeout -k 10 120 python scripts/ps_timing.py build/variants/ps_t.so --batch 512 || exit 1
timeout -k 10 120 python scripts/ps_timing.py build/variants/ps_t.so --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
