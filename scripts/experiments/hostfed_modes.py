#!/usr/bin/env python3
"""Host-fed step schedules (experiment harness): frames from pinned host memory, results back to
pinned host memory, for the c3 step (640x480, B frames, 1000 kp, SearchForInitialization on the
consecutive pairs).  Modes:
  base    H2D / compute / D2H on three streams, double-buffered (bench.py's host_fed)
  chunks  the same with the H2D split into N chunk copies
  onecopy H2D and D2H on one copy stream (one ordered DMA queue)
Prints ms per step and frames/s for each."""
import sys
import time
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import orbslam_jpminipc_amd as orb  # noqa: E402

B, W, H, NF = 512, 640, 480, 1000
frames = orb.synth_stream(W, H, stream=0, first=0, count=B)
ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
matcher = orb.ORBmatcher(0.9, True)
cap = ext.max_keypoints
f1 = torch.arange(B - 1, dtype=torch.int32, device="cuda")
f2 = f1 + 1
h_in = torch.from_numpy(frames).pin_memory()
d_in = [torch.empty_like(h_in, device="cuda") for _ in range(2)]
d_out = [(torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda"), torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda"),
          torch.empty((B,), dtype=torch.int32, device="cuda")) for _ in range(2)]
h_out = [(torch.empty((B, cap, 28), dtype=torch.uint8).pin_memory(), torch.empty((B, cap, 32), dtype=torch.uint8).pin_memory(),
          torch.empty((B,), dtype=torch.int32).pin_memory(), torch.empty((B - 1, cap), dtype=torch.int32).pin_memory(),
          torch.empty((B - 1,), dtype=torch.int32).pin_memory()) for _ in range(2)]
s_h2d, s_comp, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()


def run(mode, nchunks=4, steps=10, warm=2):
    ev_h2d = [torch.cuda.Event() for _ in range(2)]
    ev_comp = [torch.cuda.Event() for _ in range(2)]
    ev_d2h = [torch.cuda.Event() for _ in range(2)]
    s_out = s_h2d if mode == "onecopy" else s_d2h
    d_m = [None, None]

    def issue(t):
        i = t % 2
        with torch.cuda.stream(s_h2d):
            if t >= 2:
                s_h2d.wait_event(ev_comp[i])
            if mode == "chunks":
                for c in range(nchunks):
                    a, b = c * B // nchunks, (c + 1) * B // nchunks
                    d_in[i][a:b].copy_(h_in[a:b], non_blocking=True)
            else:
                d_in[i].copy_(h_in, non_blocking=True)
            ev_h2d[i].record(s_h2d)
        with torch.cuda.stream(s_comp):
            s_comp.wait_event(ev_h2d[i])
            if t >= 2:
                s_comp.wait_event(ev_d2h[i])
            kps, desc, cnt = d_out[i]
            ext.extract_batch_device(d_in[i], kps, desc, cnt, stream=s_comp)
            d_m[i] = matcher.search_for_initialization_batch_device(kps, desc, cnt, f1, f2, W, H, 100, stream=s_comp)
            ev_comp[i].record(s_comp)
        with torch.cuda.stream(s_out):
            s_out.wait_event(ev_comp[i])
            for dst, src in zip(h_out[i], (*d_out[i], *d_m[i])):
                dst.copy_(src, non_blocking=True)
            ev_d2h[i].record(s_out)

    for t in range(warm):
        issue(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        issue(t)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{mode:8s} chunks={nchunks if mode == 'chunks' else 1}: {dt * 1e3:.3f} ms/step, {B / dt:.0f} frames/s", flush=True)


for m in ("base", "chunks", "onecopy", "base"):
    run(m)
run("chunks", nchunks=16)
