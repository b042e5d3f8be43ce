#!/usr/bin/env python3
"""Experiment harness: frames/s of the bench step (B frames extract + B-1 consecutive-pair
SearchForInitialization) through FrontEndPipeline for several stream counts."""
import argparse
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import orbslam_jpminipc_amd as orb  # noqa: E402
from orbslam_jpminipc_amd.pipeline import FrontEndPipeline  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3, 4, 6, 8])
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
W, H, B = 640, 480, a.batch
frames = torch.from_numpy(orb.synth_stream(W, H, stream=0, first=0, count=B)).cuda()
st = torch.cuda.Stream()
for S in a.streams:
    p = FrontEndPipeline(1000, 1.2, 8, 1, 20, device=0, max_batch=B, n_streams=S)
    cap = p.max_keypoints
    k = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    c = torch.empty((B,), dtype=torch.int32, device="cuda")
    m = torch.empty((B - 1, cap), dtype=torch.int32, device="cuda")
    n = torch.empty((B - 1,), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        p.run(frames, k, d, c, m, n, stream=st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        p.run(frames, k, d, c, m, n, stream=st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"S={S}: {B / dt:.0f} frames/s ({dt * 1e3:.3f} ms/step), matches/pair {n.float().mean().item():.2f}",
          flush=True)
    p.close()
