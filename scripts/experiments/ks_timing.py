#!/usr/bin/env python3
"""Per-level, per-phase s_memrealtime sums of k_select from a -DKS_TIMING=1 build (experiment
harness).  Usage: ks_timing.py LIB.so [W H NF B]; prints, per level, the mean workgroup time of
each phase in us (100 MHz realtime clock) and the mean survivors per workgroup."""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

_native.HIP_LIB_PATH = pathlib.Path(sys.argv[1]).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

W, H, NF, B = (int(x) for x in (sys.argv[2:6] if len(sys.argv) >= 6 else (1241, 376, 2000, 512)))
frames = orb.synth_stream(W, H, stream=0, first=0, count=B)
d = torch.from_numpy(frames).cuda()
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
k, de, c = ext.extract_batch_device(d)
torch.cuda.synchronize()
fn = orb.hip_lib().orb_debug_ks_timing
fn.argtypes = [ctypes.c_void_p]
out = (ctypes.c_ulonglong * (16 * 8))()
fn(out)
for _ in range(3):
    ext.extract_batch_device(d, k, de, c)
torch.cuda.synchronize()
fn(out)
names = ["counts", "book", "sort", "cellretain", "lvlretain", "out"]
print(f"{W}x{H} nf={NF} B={B}: k_select mean us per workgroup (realtime clock 100 MHz)")
for lv in range(8):
    row = out[lv * 8: lv * 8 + 8]
    n = row[7]
    if not n:
        continue
    print(lv, {nm: round(row[i] / n / 100, 2) for i, nm in enumerate(names)}, "M", round(row[6] / n, 1), "wgs", n)
