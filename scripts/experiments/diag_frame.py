#!/usr/bin/env python3
"""Diagnose a GPU-vs-oracle mismatch on one synthetic frame (experiment harness): per-level
cell counts, keypoint fields that differ, descriptor rows that differ."""
import ctypes
import sys
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orbslam_jpminipc_amd as orb  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

W, H, NF = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (640, 480, 1000)))
img = orb.synth_stream(W, H, stream=0, first=0, count=1)[0]
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0)
ora = Oracle(NF, 1.2, 8, 1, 20)
kg, dg = ext(img)
ko, do = ora.extract(img)
lib = orb.hip_lib()
for l in range(8):
    cnt = np.zeros(4096, np.int32)
    n = lib.orb_debug_cell_counts(ext._h, 0, l, cnt.ctypes.data_as(ctypes.c_void_p), 4096)
    oc = ora.cell_counts(l).reshape(-1)
    if not np.array_equal(cnt[:n], oc):
        print("level", l, "cell counts differ", cnt[:n].tolist(), oc.tolist())
print("n", len(kg), len(ko))
m = min(len(kg), len(ko))
for f in kg.dtype.names:
    d = np.nonzero(kg[f][:m] != ko[f][:m])[0]
    if len(d):
        print(f, len(d), "first", d[:5], kg[d[:3]], ko[d[:3]])
rows = np.nonzero((dg[:m] != do[:m]).any(1))[0]
print("desc rows differ", len(rows), rows[:10])
for i in rows[:5]:
    print(" kp", ko[i], "bits", np.unpackbits(dg[i] ^ do[i]).nonzero()[0][:10])
