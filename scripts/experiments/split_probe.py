#!/usr/bin/env python3
"""Concurrency probe (experiment harness): the c3 bench step (extract 512 frames +
SearchForInitialization on the 511 consecutive pairs) as one batch on one stream, against the
batch split into S sub-batches extracted concurrently on S streams by S extractors (each with
its own workspace) into views of the same outputs, then one matcher pass over all pairs.
Checks that the outputs agree and prints ms per step of each.  Usage: split_probe.py [W H NF B]"""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import orbslam_jpminipc_amd as orb  # noqa: E402

W, H, NF, B = (int(x) for x in (sys.argv[1:5] if len(sys.argv) >= 5 else (640, 480, 1000, 512)))
frames = orb.synth_stream(W, H, stream=0, first=0, count=B)
d_imgs = torch.from_numpy(frames).cuda()
matcher = orb.ORBmatcher(0.9, True)
f1 = torch.arange(B - 1, dtype=torch.int32, device="cuda")
f2 = f1 + 1


def run(S, steps=30, warm=5, offset=False):
    exts = [orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B // S) for _ in range(S)]
    cap = exts[0].max_keypoints
    d_kps = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(S)]
    ev = [torch.cuda.Event() for _ in range(S)]
    s0 = streams[0]
    h = B // S

    ev_pyr = [torch.cuda.Event() for _ in range(S)]

    def step():
        for i, (e, s) in enumerate(zip(exts, streams)):
            # offset: sub-batch i starts its pyramid when sub-batch i-1's pyramid is done, so a
            # pyramid overlaps the previous sub-batch's detection and descriptors
            if i:
                s.wait_event(ev_pyr[i - 1] if offset else ev_start)
            args = (d_imgs[i * h:(i + 1) * h], d_kps[i * h:(i + 1) * h], d_desc[i * h:(i + 1) * h],
                    d_cnt[i * h:(i + 1) * h])
            if offset:
                e.set_phases(1)
                e.extract_batch_device(*args, stream=s)
                ev_pyr[i].record(s)
                e.set_phases(2)
                e.extract_batch_device(*args, stream=s)
                e.set_phases(3)
            else:
                e.extract_batch_device(*args, stream=s)
            ev[i].record(s)
        for i in range(1, S):
            s0.wait_event(ev[i])
        m12, nm = matcher.search_for_initialization_batch_device(d_kps, d_desc, d_cnt, f1, f2, W, H, 100, stream=s0)
        ev_start.record(s0)
        return m12

    ev_start = torch.cuda.Event()
    ev_start.record(s0)
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m12 = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return ms, d_kps.clone(), d_desc.clone(), d_cnt.clone(), m12.clone()


ref = run(1)
print(f"{W}x{H} nf={NF} B={B}: 1 stream {ref[0]:.3f} ms/step ({B / ref[0] * 1e3:.0f} frames/s)")
for S, off in ((2, False), (2, True), (4, True)):
    r = run(S, offset=off)
    same = all(torch.equal(a, b) for a, b in zip(ref[1:], r[1:]))
    print(f"  {S} streams{' offset' if off else ''} {r[0]:.3f} ms/step ({B / r[0] * 1e3:.0f} frames/s), "
          f"outputs identical: {same}")
