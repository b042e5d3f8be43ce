#!/bin/bash
# Round-4 A/B session: parity of the in-tree build (core parity file + the c3 / c4 bench
# batches), rocprofv3 kernel means of the in-tree build vs build/variants/*.so at c3 and c4,
# and one SQ instruction-mix PMC pass of the in-tree extraction at c3.
# Usage: bash scripts/r04_ab.sh TAG VARIANT...
set -o pipefail
TAG=${1:-r04_ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_bench_batch_full_parity" "tests/test_gpu_configs.py::test_bench_batch_c4_full_parity" -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed rc=$?"; tail -30 $OUT/parity.log; exit 1; }
tail -3 $OUT/parity.log
bash scripts/variant_kstats.sh $TAG/c3 "$@" -- --batch 512 || exit 1
bash scripts/variant_kstats.sh $TAG/c4 "$@" -- --batch 512 --width 1241 --height 376 --nfeatures 2000 || exit 1
bash scripts/variant_kstats.sh $TAG/c5 "$@" -- --batch 512 --width 1280 --height 720 --nfeatures 2500 || exit 1
cat $OUT/c3/kstats.txt $OUT/c4/kstats.txt $OUT/c5/kstats.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/pmc -o run --output-format csv -- python scripts/stage_times.py --batch 512 --steps 3 > $OUT/pmc.log 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
python3 - $OUT/pmc <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k in sorted(acc):
    if not k.startswith("k_"): continue
    d = {c: v / n[k] for c, v in acc[k].items()}
    w = d.get("SQ_WAVES", 1)
    print(k, "launches", n[k], {c: round(v / w, 1) for c, v in sorted(d.items()) if c != "SQ_WAVES"}, "waves", w)
PY
if [ -f build/variants/krtiming.so ]; then
  timeout -k 10 120 python scripts/kr_timing.py build/variants/krtiming.so 1241 376 2000 512 > $OUT/kr_c4.txt 2>&1 || exit 1
  timeout -k 10 180 python scripts/kr_timing.py build/variants/krtiming.so 1280 720 2500 512 > $OUT/kr_c5.txt 2>&1 || exit 1
  cat $OUT/kr_c4.txt $OUT/kr_c5.txt
fi
if [ -f build/variants/kftiming.so ]; then
  timeout -k 10 120 python scripts/kf_timing.py build/variants/kftiming.so > $OUT/kf_c3.txt 2>&1 || exit 1
  cat $OUT/kf_c3.txt
fi
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES -d $OUT/pmc2 -o run --output-format csv -- python scripts/stage_times.py --batch 512 --steps 3 > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed rc=$?"; exit 1; }
python3 - $OUT/pmc2 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k in sorted(acc):
    if not k.startswith("k_"): continue
    d = {c: v / n[k] for c, v in acc[k].items()}
    w = d.get("SQ_WAVES", 1)
    tot = d.get("SQ_WAIT_ANY", 0) + d.get("SQ_WAIT_INST_ANY", 0) + d.get("SQ_ACTIVE_INST_ANY", 0)
    print(k, {c: round(v / w, 1) for c, v in sorted(d.items()) if c != "SQ_WAVES"},
          {"wait": round(d.get("SQ_WAIT_ANY", 0) / max(tot, 1), 3), "issue_stall": round(d.get("SQ_WAIT_INST_ANY", 0) / max(tot, 1), 3),
           "active": round(d.get("SQ_ACTIVE_INST_ANY", 0) / max(tot, 1), 3)})
PY
