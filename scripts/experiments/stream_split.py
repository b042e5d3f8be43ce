#!/usr/bin/env python3
"""Experiment: the bench workload (B frames extract + B-1 pair matches) split over S
independent extractor handles on S HIP streams (frames b*S/.. per stream), vs one stream.
Prints frames/s for S = 1, 2, 3, 4."""
import sys
import time
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import orbslam_jpminipc_amd as orb  # noqa: E402

W, H, B = 640, 480, 256
frames = torch.from_numpy(orb.synth_stream(W, H, stream=0, first=0, count=B)).cuda()
for S in (1, 2, 3, 4):
    chunks = [(B * i) // S for i in range(S + 1)]
    ctx = []
    for i in range(S):
        n = chunks[i + 1] - chunks[i]
        e = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=n)
        cap = e.max_keypoints
        st = torch.cuda.Stream()
        k = torch.empty((n, cap, 28), dtype=torch.uint8, device="cuda")
        d = torch.empty((n, cap, 32), dtype=torch.uint8, device="cuda")
        c = torch.empty((n,), dtype=torch.int32, device="cuda")
        f1 = torch.arange(0, n - 1, dtype=torch.int32, device="cuda")
        ctx.append((e, st, frames[chunks[i]:chunks[i + 1]], k, d, c, f1, f1 + 1))
    m = orb.ORBmatcher(0.9, True)

    def step():
        for e, st, fr, k, d, c, f1, f2 in ctx:
            with torch.cuda.stream(st):
                e.extract_batch_device(fr, k, d, c, stream=st)
                m.search_for_initialization_batch_device(k, d, c, f1, f2, W, H, 100, stream=st)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    N = 20
    for _ in range(N):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"S={S}: {B * N / dt:.0f} frames/s  ({dt / N * 1e3:.3f} ms/step)", flush=True)
