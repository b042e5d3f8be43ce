"""The overlapped front-end pipeline (csrc/orb_pipeline.hip) equals the serial path:
extract_batch_device + search_for_initialization_batch_device on one stream, bit for bit."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.pipeline import FrontEndPipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,S", [(9, 4), (3, 8), (8, 1), (17, 3)])
def test_pipeline_equals_serial_path(B, S):
    import torch

    W, H = 640, 480
    frames = torch.from_numpy(orb.synth_stream(W, H, stream=60 + B, first=0, count=B)).cuda()
    pipe = FrontEndPipeline(1000, 1.2, 8, 1, 20, device=0, max_batch=B, n_streams=S)
    cap = pipe.max_keypoints
    k = torch.zeros((B, cap, 28), dtype=torch.uint8, device="cuda")
    d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    c = torch.zeros((B,), dtype=torch.int32, device="cuda")
    m12 = torch.full((max(B - 1, 1), cap), -7, dtype=torch.int32, device="cuda")
    nm = torch.full((max(B - 1, 1),), -7, dtype=torch.int32, device="cuda")
    pipe.run(frames, k, d, c, m12, nm)
    torch.cuda.synchronize()
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    k2, d2, c2 = ext.extract_batch_device(frames)
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    m2, n2 = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(k2, d2, c2, f1, f1 + 1, W, H, 100)
    torch.cuda.synchronize()
    assert torch.equal(c, c2)
    for b in range(B):
        n = int(c[b])
        assert torch.equal(k[b, :n], k2[b, :n]) and torch.equal(d[b, :n], d2[b, :n])
    assert torch.equal(nm[:B - 1], n2)
    for p in range(B - 1):
        n = int(c[p])
        assert torch.equal(m12[p, :n], m2[p, :n])
