#!/usr/bin/env python3
"""Per-stage HIP-event times of the extraction pipeline for one liborb_hip.so build.

Experiment harness (not the product path): `stage_times.py [LIB.so] [--batch B]` loads the
given library build (default: the in-tree one) and prints ms per launch of every stage over
the bench workload (B synthetic 640x480 frames, ORBextractor(1000, 1.2, 8, FAST, 20)).
"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("lib", nargs="?")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--height", type=int, default=480)
ap.add_argument("--nfeatures", type=int, default=1000)
a = ap.parse_args()

import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

if a.lib:
    _native.HIP_LIB_PATH = pathlib.Path(a.lib).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

B = a.batch
frames = orb.synth_stream(a.width, a.height, stream=0, first=0, count=B)
d = torch.from_numpy(frames).cuda()
ext = orb.ORBextractor(a.nfeatures, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
cap = ext.max_keypoints
k = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
de = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
c = torch.empty((B,), dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for _ in range(3):
    ext.extract_batch_device(d, k, de, c, stream=s)
torch.cuda.synchronize()
ext.profile_enable(True)
for _ in range(a.steps):
    ext.extract_batch_device(d, k, de, c, stream=s)
torch.cuda.synchronize()
prof = ext.profile_read()
out = {n: round(ms / max(l, 1), 4) for n, (ms, l) in prof.items()}
# SearchForInitialization on the B-1 consecutive pairs of the batch (the bench step's matcher)
if B > 1:
    m = orb.ORBmatcher(0.9, True)
    f1 = torch.arange(B - 1, dtype=torch.int32, device="cuda")
    f2 = f1 + 1
    for _ in range(2):
        m.search_for_initialization_batch_device(k, de, c, f1, f2, a.width, a.height, 100, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.steps):
        m.search_for_initialization_batch_device(k, de, c, f1, f2, a.width, a.height, 100, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    out["k_match_init"] = round(e0.elapsed_time(e1) / a.steps, 4)
out["lib"] = os.path.basename(str(_native.HIP_LIB_PATH))
print(json.dumps(out))
