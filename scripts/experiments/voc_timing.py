"""Time ORBVocabulary.transform_batch_device (Frame::ComputeBoW for a batch, Frame.cc:280-287)
on an ORBvoc-shaped tree (k=10, L=6, 1 111 111 nodes, random) over the extractor's own
output for B frames of the c3 workload (640x480, 1000 features).  One JSON line on stdout.
Usage: python scripts/voc_timing.py [--batch 512] [--iters 20] [--levelsup 4]"""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import orbslam_jpminipc_amd as orb  # noqa: E402


def random_tree(k, L, seed):
    """Complete k-ary tree of depth L in file order (parents before children), random node
    descriptors and leaf weights (as tests/vocab_util.random_vocabulary)."""
    rng = np.random.default_rng(seed)
    n = sum(k ** d for d in range(1, L + 1))
    parent = np.zeros(n, np.int32)
    width, pos = 1, 0  # the previous level's nodes: prev_first .. prev_first + width - 1 (root 0)
    prev_first = 0
    for d in range(1, L + 1):
        parent[pos:pos + width * k] = np.repeat(np.arange(prev_first, prev_first + width, dtype=np.int32), k)
        prev_first = pos + 1
        pos += width * k
        width *= k
    leaf = np.zeros(n, np.uint8)
    leaf[n - k ** L:] = 1
    desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    weight = np.where(leaf > 0, rng.uniform(0.0, 3.0, size=n), 0.0)
    return parent, leaf, desc, weight

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--levelsup", type=int, default=4)
a = ap.parse_args()

t0 = time.time()
gv = orb.ORBVocabulary.from_arrays(10, 6, 0, 0, *random_tree(10, 6, 106))
t_build = time.time() - t0
B = a.batch
ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
imgs = torch.from_numpy(orb.synth_stream(640, 480, stream=0, first=0, count=B)).cuda()  # B distinct frames
d_kps, d_desc, d_counts = ext.extract_batch_device(imgs)
out = gv.transform_batch_device(d_desc, d_counts, a.levelsup)
s = torch.cuda.current_stream()
for _ in range(3):
    gv.transform_batch_device(d_desc, d_counts, a.levelsup, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(a.iters):
    gv.transform_batch_device(d_desc, d_counts, a.levelsup, out=out)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
nfeat = int(d_counts.sum().item())
print(json.dumps({"what": "ORBVocabulary.transform_batch_device, k=10 L=6 (1111111 nodes)", "batch": B,
                  "features": nfeat, "levelsup": a.levelsup, "ms_per_batch": round(ms, 4),
                  "us_per_frame": round(1000 * ms / B, 3), "frames_per_s": round(1000 * B / ms, 1),
                  "features_per_s": round(1000 * nfeat / ms), "vocab_build_s": round(t_build, 2)}))
