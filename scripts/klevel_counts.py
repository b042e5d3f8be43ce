#!/usr/bin/env python3
"""k_level FAST-queue volume over one bench batch (experiment harness, not the product path).

Usage: klevel_counts.py LIB.so  — LIB built with -DKL_COUNT=1 (scripts/build_variant.sh).
Prints lane-rows queued, pixels expanded and corners per frame.
"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

_native.HIP_LIB_PATH = pathlib.Path(sys.argv[1]).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

B = 256
frames = orb.synth_stream(640, 480, stream=0, first=0, count=B)
d = torch.from_numpy(frames).cuda()
ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
cap = ext.max_keypoints
k = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
de = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
c = torch.empty((B,), dtype=torch.int32, device="cuda")
lib = orb.hip_lib()
out = np.zeros(3, np.uint64)
ext.extract_batch_device(d, k, de, c)
torch.cuda.synchronize()
lib.orb_debug_klevel_counts(out.ctypes.data)
ext.extract_batch_device(d, k, de, c)
torch.cuda.synchronize()
lib.orb_debug_klevel_counts(out.ctypes.data)
print({"lane_rows_per_frame": int(out[0]) / B, "pixels_per_frame": int(out[1]) / B, "corners_per_frame": int(out[2]) / B})
