#!/usr/bin/env python3
"""Timing-only ablation (WRONG OUTPUT; experiment harness): k_orient_desc as it would run if a
blurred copy of every level were already in LDS -- no row pass on the matrix cores and each
rBRIEF sample one LDS dword read instead of the column pass (four v_dot2 over row pairs, the tap
selection by row parity).  Bounds what a per-level blur (option A) could save
in k_orient_desc, before the cost of producing the blurred levels.
Usage: od_preblur_ablation.py NAME  ->  build/variants/NAME.so"""
import subprocess
import sys

reps = [
    ("    if (active) {\n        const int r16 = lane & 15, h4 = lane >> 4;",
     "    if (false) {\n        const int r16 = lane & 15, h4 = lane >> 4;"),
    ("        const uint32_t T = dot2u(hq[3 * OD_HN], t3, dot2u(hq[2 * OD_HN], t2, dot2u(hq[OD_HN], t1, dot2u(hq[0], t0, 0u))));",
     "        const uint32_t T = hq[0] << 8; (void)t0; (void)t1; (void)t2; (void)t3;"),
]
args = ["python3", "scripts/ablation_variant.py", sys.argv[1]]
for a, b in reps:
    args += [a, b]
sys.exit(subprocess.call(args))
