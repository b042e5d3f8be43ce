#!/bin/bash
# Per-kernel mean durations (rocprofv3 --kernel-trace --stats) of stage_times.py for the in-tree
# library and each build/variants/NAME.so given.
# Usage (via gpurun): bash scripts/variant_kstats.sh TAG NAME... [-- stage_times args]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
libs="intree"; extra=""
while [ $# -gt 0 ]; do if [ "$1" = "--" ]; then shift; extra="$@"; break; fi; libs="$libs $1"; shift; done
for v in $libs; do
  lib=""; [ "$v" = "intree" ] || lib=build/variants/$v.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ks_$v -o run --output-format csv -- python scripts/stage_times.py $lib $extra > $OUT/ks_$v.log 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  python3 - "$OUT/ks_$v" "$v" >> $OUT/kstats.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print(sys.argv[2], {k: round(v, 1) for k, v in rows.items() if k.startswith("k_")})
PY
done
