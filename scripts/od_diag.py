#!/usr/bin/env python3
"""Descriptor-difference diagnosis (experiment harness): extract the frames of
test_extract_parity_configs[W-H-nf] with the library named by ORB_HIP_LIB (or the in-tree one)
and the oracle, and print, per differing descriptor row, the keypoint, its window alignment and
the differing rBRIEF tests (test i = pattern points 2i, 2i+1; lane i // 4 of k_orient_desc).
Usage: od_diag.py [W H nf [reps]]; ORB_DIAG_SELF=1 compares every repetition with the first
GPU run of the frame instead of the oracle (run-to-run nondeterminism of wrong-output builds)."""
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orbslam_jpminipc_amd as orb  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

W, H, NF = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (640, 480, 2000)))
REPS = int(sys.argv[4]) if len(sys.argv) >= 5 else 6
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0)
ora = Oracle(NF, 1.2, 8, 1, 20)
tot = 0
for fi, img in enumerate(orb.synth_stream(W, H, stream=3, first=0, count=3)):
    for rep in range(REPS):
        kg, dg = ext(img)
        if hasattr(orb.hip_lib(), "orb_variant_odp"):  # probe builds: pattern registers that differ
            import ctypes

            buf = np.zeros(8 * 512, np.uint32)
            fn = orb.hip_lib().orb_variant_odp
            fn.restype = ctypes.c_int
            nprobe = fn(buf.ctypes.data_as(ctypes.c_void_p), 512)
            for i in range(min(nprobe, 16)):
                o = buf[8 * i: 8 * i + 8]
                got = o[3:7].view(np.float32)
                print(f"  probe: wave {o[0] >> 16} lane {(o[0] >> 8) & 255} q {o[0] & 255} slot {o[1]} frame {o[2]} "
                      f"block {o[7]} got {got.tolist()} bits {[hex(x) for x in o[3:7]]}")
            if nprobe:
                print(f"  probe records: {nprobe}")
        ko, do = ora.extract(img)
        if os.environ.get("ORB_DIAG_SELF"):
            if rep == 0:
                ko, do = kg.copy(), (dg.copy() if dg is not None else None)
                first = (ko, do)
            else:
                ko, do = first
        if kg.tobytes() != ko.tobytes():
            print(f"frame {fi} rep {rep}: keypoints differ")
            continue
        if dg is None:
            continue
        rows = np.nonzero((dg != do).any(axis=1))[0]
        tot += len(rows)
        print(f"frame {fi} rep {rep}: {len(rows)} rows differ of {len(dg)}")
        for r in rows[:8]:
            k = kg[r]
            lvl = int(k["octave"]) if k.dtype.names else int(k[5])
            bits = np.unpackbits(dg[r] ^ do[r], bitorder="little")
            tests = np.nonzero(bits)[0]
            print(f"  row {r} kp {k} level {lvl} tests {tests.tolist()}")
print("total differing rows", tot)
