#!/bin/bash
# round 5 call X: the zero-copy SearchForInitialization host call (default now) -- -m gpu suite,
# the per-call breakdown and the C++ latency harness
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_x
mkdir -p $OUT build
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
hipcc --offload-arch=gfx950 -O2 -w -o build/sfi_breakdown scripts/sfi_breakdown.cpp -Lorbslam_jpminipc_amd -lorb_hip -lsynth -Wl,-rpath,'$ORIGIN/../orbslam_jpminipc_amd' || exit 1
timeout -k 10 120 ./build/sfi_breakdown > $OUT/bd.json || exit 1
python -c "import pathlib, subprocess, __graft_entry__ as g; subprocess.check_call(g.LATENCY_CMD(pathlib.Path('build/latency_gpu').resolve()))" || exit 1
timeout -k 10 120 ./build/latency_gpu 640 480 1000 200 > $OUT/latency.json || exit 1
cat $OUT/bd.json $OUT/latency.json
