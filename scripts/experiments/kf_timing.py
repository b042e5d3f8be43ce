#!/usr/bin/env python3
"""Per-phase s_memtime sums of k_fast from a -DKF_TIMING=1 build (experiment harness)."""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from orbslam_jpminipc_amd import _native  # noqa: E402

_native.HIP_LIB_PATH = pathlib.Path(sys.argv[1]).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402

B = 512
frames = orb.synth_stream(640, 480, stream=0, first=0, count=B)
d = torch.from_numpy(frames).cuda()
ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
k, de, c = ext.extract_batch_device(d)
torch.cuda.synchronize()
lib = orb.hip_lib()
fn = lib.orb_debug_kf_timing
fn.argtypes = [ctypes.c_void_p]
out = (ctypes.c_ulonglong * 6)()
fn(out)
for _ in range(3):
    ext.extract_batch_device(d, k, de, c)
torch.cuda.synchronize()
fn(out)
waves = out[5]
names = ["stage", "rows", "drain", "barrier", "nms"]
print({n: round(out[i] / waves, 1) for i, n in enumerate(names)}, "waves", waves)
