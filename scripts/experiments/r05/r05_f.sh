#!/bin/bash
# round 5 call F: per-call latency in C++ (build/latency_gpu) and its kernel trace
set -o pipefail
mkdir -p gpurun_out/r05_f
export TMPDIR=/tmp
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 > gpurun_out/r05_f/lat_c3.json || exit 1
cat gpurun_out/r05_f/lat_c3.json
timeout -k 10 120 ./build/latency_gpu 1241 376 2000 200 > gpurun_out/r05_f/lat_c4.json || exit 1
cat gpurun_out/r05_f/lat_c4.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_f/prof -o run --output-format csv -- ./build/latency_gpu 640 480 1000 50 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05_f/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
