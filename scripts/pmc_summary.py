#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from the rocprofv3 PMC passes of scripts/pmc_pass.sh.

Usage: pmc_summary.py gpurun_out/TAG [--json OUT] [--width W --height H --batch B --nfeatures N]
(bench.py reads profiles/pmc_<workload>.json for the roofline's `traffic`)

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0 request counters, MI355X_MICROARCH.md
§HBM).  The guide's ×2 FETCH correction holds for 16-B/lane streaming loads; it is measured in
the same run on k_pyr0, which reads exactly the B input frames (B·W·H bytes, evicted from the
256 MiB Infinity Cache by the ~0.6 GB every step writes) with 16-B loads, and applied to the
16-B-load kernels (k_pyr0, k_pyr_resize, k_fast's tile staging, k_orient_desc's patch
windows).  The dword-load kernels use the factor measured the
same way when k_pyr0 still loaded dwords (r01_v16: 1.353).  WRITE_SIZE is taken as is (exact
for streaming stores per the guide).
"""
import argparse
import csv
import glob
import json
from collections import defaultdict


WIDE_LOADS = {"k_pyr0", "k_pyr_stream", "k_pyr_resize", "k_fast", "k_orient_desc", "k_rerun",  # k_rerun: round 4
              "k_voc_descend", "k_bow_pairs"}  # round 5: 16-B child-descriptor / descriptor loads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--dword-factor", type=float, default=1.3532485621757968,
                    help="FETCH_SIZE calibration of dword-per-lane loads: measured on k_pyr0 when it "
                         "loaded dwords (profiles/r01_v16_pmc.json)")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{a.root}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "")
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()
            if not k.startswith("__amd") and "elementwise" not in k and "at::" not in k}
    known = a.batch * a.width * a.height
    # the kernel that reads exactly the B input frames from HBM: k_pyr0, or k_pyr_stream (whose
    # other reads, the shared column / row tables, are L2-resident)
    ck = "k_pyr0" if "k_pyr0" in mean else "k_pyr_stream"
    cal = known / (mean[ck]["FETCH_SIZE"] * 1024.0) if ck in mean else None
    out = {"source": a.root.rstrip("/").split("/")[-1],
           "workload": {"width": a.width, "height": a.height, "batch": a.batch, "nfeatures": a.nfeatures},
           "read_calibration": {"kernel": ck, "known_read_bytes": known, "factor": cal,
                                "applies_to": sorted(WIDE_LOADS), "dword_factor": a.dword_factor,
                                "dword_factor_source": "r01_v16_pmc (k_pyr0 with dword loads)"},
           "per_launch": {}}
    for k, d in sorted(mean.items()):
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        # WIDE_LOADS load 16 B per lane (calibrated here on k_pyr0's known read, the guide's x2);
        # the other kernels load dwords (the r01_v16 dword calibration)
        rd = d["FETCH_SIZE"] * 1024.0 * ((cal or 1.0) if k in WIDE_LOADS else a.dword_factor)
        wr = d["WRITE_SIZE"] * 1024.0
        out["per_launch"][k] = {"fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"], "read_bytes": rd,
                                "write_bytes": wr, "hbm_bytes": rd + wr,
                                **{c: v for c, v in d.items() if c.startswith("SQ_")}}
        print(f"{k:16s} read {rd / 1e6:10.2f} MB  write {wr / 1e6:10.2f} MB  per launch")
    print(f"read calibration factor ({ck}): {cal}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
