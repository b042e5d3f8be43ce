#!/bin/bash
# Repeated-extraction race screen of the in-tree build (scripts/od_diag.py: 3 frames x 6
# repetitions against the oracle) at the four parity configurations.
set -o pipefail
OUT=gpurun_out/${1:-r04_race}
mkdir -p $OUT
for cfg in "640 480 1000" "640 480 2000" "1241 376 2000" "1280 720 2500"; do
  n=$(echo $cfg | tr ' ' _)
  timeout -k 10 300 python scripts/od_diag.py $cfg > $OUT/$n.txt 2>&1 || { echo "diag $cfg rc=$?"; tail -5 $OUT/$n.txt; exit 1; }
  echo "$cfg: $(tail -1 $OUT/$n.txt)"
done
