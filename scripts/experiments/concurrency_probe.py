"""Experiment harness: the bench step (extraction of B frames + SearchForInitialization of the
B-1 consecutive pairs) on one stream vs FrontEndPipeline cut into S chunk streams.
Prints ms per step for each S.  Usage: concurrency_probe.py [--batch 512] [--width W ...]"""
import argparse
import json
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--height", type=int, default=480)
ap.add_argument("--nfeatures", type=int, default=1000)
ap.add_argument("--streams", default="1,2,3,4,8")
ap.add_argument("--lib", default=None, help="a liborb_hip.so build to load instead of the in-tree one")
a = ap.parse_args()
if a.lib:
    from orbslam_jpminipc_amd import _native  # noqa: E402

    _native.HIP_LIB_PATH = pathlib.Path(a.lib).resolve()
import orbslam_jpminipc_amd as orb  # noqa: E402
from orbslam_jpminipc_amd.pipeline import FrontEndPipeline  # noqa: E402

B, W, H, NF = a.batch, a.width, a.height, a.nfeatures
frames = torch.from_numpy(orb.synth_stream(W, H, stream=0, first=0, count=B)).cuda()
res = {}
for S in [int(x) for x in a.streams.split(",")]:
    pipe = FrontEndPipeline(NF, 1.2, 8, 1, 20, device=0, max_batch=B, n_streams=S)
    cap = pipe.max_keypoints
    k = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    c = torch.empty((B,), dtype=torch.int32, device="cuda")
    m = torch.empty((B - 1, cap), dtype=torch.int32, device="cuda")
    n = torch.empty((B - 1,), dtype=torch.int32, device="cuda")
    for _ in range(3):
        pipe.run(frames, k, d, c, m, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        pipe.run(frames, k, d, c, m, n)
    torch.cuda.synchronize()
    res[S] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
    pipe.close()
print(json.dumps({"workload": [W, H, NF, B], "lib": a.lib, "ms_per_step_by_streams": res}))
