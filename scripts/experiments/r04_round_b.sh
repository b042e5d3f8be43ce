#!/bin/bash
# c5 bench + rocprof + PMC, clean c3 / c4 kernel statistics (no host-fed leg), host-fed copy modes
set -o pipefail
TAG=${1:-r04_v4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PMC=1 bash scripts/bench_all.sh $TAG c5 || exit $?
for wl in c3 c4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$wl -o run --output-format csv -- python bench.py --workload $wl --cpu-frames 0 --latency 0 --host-fed 0 > $OUT/prof_$wl.log 2>&1 || { echo "rocprof $wl rc=$?"; exit 1; }
done
timeout -k 10 300 python scripts/hostfed_modes.py > $OUT/modes_default.txt 2>&1 || { echo "modes rc=$?"; exit 1; }
HSA_ENABLE_SDMA=1 timeout -k 10 300 python scripts/hostfed_modes.py > $OUT/modes_sdma1.txt 2>&1 || { echo "modes sdma rc=$?"; exit 1; }
cat $OUT/summary.txt $OUT/modes_default.txt $OUT/modes_sdma1.txt
