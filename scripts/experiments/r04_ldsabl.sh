#!/bin/bash
# k_orient_desc LDS bank-conflict attribution: one SQ pass (conflict cycles, LDS instructions)
# over stage_times.py for the in-tree build and each wrong-output ablation build given (one
# access site made conflict-free each), plus their kernel means.
# Usage: bash scripts/r04_ldsabl.sh TAG NAME...
set -o pipefail
TAG=${1:-r04_lds}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in intree "$@"; do
  lib=""; [ "$v" = "intree" ] || lib=build/variants/$v.so
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES -d $OUT/p_$v -o run --output-format csv -- python scripts/stage_times.py $lib --batch 512 --steps 3 > $OUT/p_$v.log 2>&1 || { echo "pmc $v failed rc=$?"; exit 1; }
  python3 - $OUT/p_$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = 0; dur = []
for r in csv.DictReader(open(f)):
    if not r["Kernel_Name"].startswith("k_orient_desc"): continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n += 1
w = acc["SQ_WAVES"]
print(sys.argv[2], "conflict cycles / wave", round(acc["SQ_LDS_BANK_CONFLICT"] / w, 1), "LDS insts / wave", round(acc["SQ_INSTS_LDS"] / w, 1), "launches", n)
PY
done
bash scripts/variant_kstats.sh $TAG/kst "$@" -- --batch 512 || exit 1
cat $OUT/kst/kstats.txt
