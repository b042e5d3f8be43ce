#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel over all passes of scripts/pmc_pass.sh."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if k.startswith("__amd") or "elementwise" in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")
