#!/usr/bin/env python3
"""k_pyr_stream phase timing (experiment harness, PS_TIMING=1 builds only): per-wave s_memtime
cycles per round in fetch issue / task loop / barrier 1 / put / barrier 2.
Usage: ps_timing.py LIB.so [--batch B] [--width W --height H --nfeatures N]"""
import argparse
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--height", type=int, default=480)
ap.add_argument("--nfeatures", type=int, default=1000)
a = ap.parse_args()
import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

_native.HIP_LIB_PATH = pathlib.Path(a.lib).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

lib = orb.hip_lib()
B = a.batch
frames = orb.synth_stream(a.width, a.height, stream=0, first=0, count=B)
d = torch.from_numpy(frames).cuda()
ext = orb.ORBextractor(a.nfeatures, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
ext.set_phases(1)
ext.extract_batch_device(d)
torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 32)()
lib.orb_debug_ps_timing(out)
k0, nr, lds = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
lib.orb_debug_pyramid_plan(ext._h, ctypes.byref(k0), ctypes.byref(nr), ctypes.byref(lds))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    ext.extract_batch_device(d)
e1.record()
torch.cuda.synchronize()
lib.orb_debug_ps_timing(out)
waves = out[5]
names = ["fetch", "tasks", "barrier1", "put", "barrier2"]
per = {n: out[i] / max(waves, 1) / max(nr.value, 1) for i, n in enumerate(names)}
print(f"{a.width}x{a.height} B={B} K0={k0.value} rounds={nr.value} lds={lds.value} "
      f"ms/launch={e0.elapsed_time(e1) / 5:.4f} waves={waves}")
print("cycles per wave per round: " + ", ".join(f"{n} {v:.0f}" for n, v in per.items()))
# per level: task cycles per builder wave per round (g_pstime[8 + l] over g_pstime[24 + l] waves)
print("task cycles per round by level: " + ", ".join(
    f"L{l} {out[8 + l] / max(out[24 + l], 1) / max(nr.value, 1):.0f} ({out[24 + l] // max(B * 5 + B, 1)} waves)"
    for l in range(8) if out[24 + l]))
print("cycles per wave total: " + ", ".join(f"{n} {out[i] / max(waves, 1):.0f}" for i, n in enumerate(names)))
print("task cycles per wave per round by level: " + ", ".join(
    f"L{l} {out[8 + l] / max(out[24 + l], 1) / max(nr.value, 1):.0f}" for l in range(8) if out[24 + l]))
