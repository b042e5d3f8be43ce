#!/usr/bin/env python3
"""k_match_init phase timing (experiment harness, KM_TIMING=1 builds only): mean per-pair
wall time of each phase (s_memrealtime, 100 MHz) for bench.py's batch of a workload.
Usage: km_timing.py LIB.so [--workload c3|c4|c5] [--per N]"""
import argparse
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--workload", default="c3")
ap.add_argument("--per", type=int, default=0, help="frames per stream (0: the bench default)")
a = ap.parse_args()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

_native.HIP_LIB_PATH = pathlib.Path(a.lib).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

W, H, NF, S = {"c3": (640, 480, 1000, 1), "c4": (1241, 376, 2000, 1), "c5": (1280, 720, 2500, 8)}[a.workload]
per = a.per or (512 if S == 1 else 128)
frames = np.concatenate([orb.synth_stream(W, H, stream=s, first=0, count=per) for s in range(S)])
B = len(frames)
lib = orb.hip_lib()
lib.orb_debug_km_timing.argtypes = [ctypes.c_void_p]
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
kps, desc, cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
f1 = torch.tensor([k * per + t for k in range(S) for t in range(per - 1)], dtype=torch.int32, device="cuda")
M = orb.ORBmatcher(0.9, True)
out = (ctypes.c_ulonglong * 8)()
for rep in range(3):
    lib.orb_debug_km_timing(out)  # reset
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    M.search_for_initialization_batch_device(kps, desc, cnt, f1, f1 + 1, W, H, 100)
    e1.record()
    torch.cuda.synchronize()
    lib.orb_debug_km_timing(out)
    P = out[5]
    print(a.workload, f"B={B} pairs={P} launch {e0.elapsed_time(e1):.4f} ms; per pair (us): " +
          " ".join(f"{n}={out[i] / P / 100:.1f}" for i, n in enumerate(["ph0", "rank", "ph1", "ph2", "ph3"])) +
          f"; queries/pair {out[6] / P:.0f} cands/pair {out[7] / P:.0f}")
