"""Stream resource hooks of the C ABI on the GPU (include/orb_abi.h):
orb_stream_create_dedicated / orb_stream_destroy (a stream with a hardware queue of its own, the
host-fed step's three streams) and orb_match_release_stream_scratch (the large-capacity
SearchForInitialization scratch kept per (device, stream)): results on such streams are
bit-exact with the oracle, and a released scratch is re-created by the next call."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.streams import dedicated_stream
from oracle_lib import search_for_initialization

pytestmark = pytest.mark.gpu


def _check_pairs(kps, desc, counts, m12, nm, W, H):
    kps_h, desc_h, cnt = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
    for p in range(len(nm)):
        n1, n2 = cnt[p], cnt[p + 1]
        k1 = orb.keypoints_from_bytes(kps_h[p], n1)
        k2 = orb.keypoints_from_bytes(kps_h[p + 1], n2)
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, desc_h[p, :n1], k2, desc_h[p + 1, :n2], W, H, prev, 0.9, True, 100)
        assert nm[p] == no
        assert np.array_equal(m12[p, :n1], m12o)


def test_dedicated_stream_extract_and_match():
    import torch

    B, W, H = 4, 640, 480
    frames = orb.synth_stream(W, H, stream=11, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    ref = ext.extract_batch_device(d)
    torch.cuda.synchronize()
    s = dedicated_stream(0)
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream())
        kps, desc, cnt = ext.extract_batch_device(d, stream=s)
        f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
        m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(kps, desc, cnt, f1, f1 + 1, W, H,
                                                                                 100, stream=s)
    s.synchronize()
    n = cnt.cpu().numpy()
    assert np.array_equal(n, ref[2].cpu().numpy())
    for b in range(B):
        assert kps[b, : n[b]].cpu().numpy().tobytes() == ref[0][b, : n[b]].cpu().numpy().tobytes()
        assert desc[b, : n[b]].cpu().numpy().tobytes() == ref[1][b, : n[b]].cpu().numpy().tobytes()
    _check_pairs(kps, desc, cnt, m12, nm, W, H)


def test_dedicated_stream_create_destroy_c_abi():
    """The C pair as a C caller uses it: create, run an extraction on it, synchronise, destroy."""
    import ctypes

    import torch

    lib = orb.hip_lib()
    h = ctypes.c_void_p()
    assert lib.orb_stream_create_dedicated(ctypes.byref(h)) == 0 and h.value
    B, W, H = 2, 640, 480
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(orb.synth_stream(W, H, stream=3, first=0, count=B)).cuda()
    ref = ext.extract_batch_device(d)
    kps = torch.empty_like(ref[0])
    desc = torch.empty_like(ref[1])
    cnt = torch.empty_like(ref[2])
    torch.cuda.synchronize()
    s = torch.cuda.ExternalStream(h.value)
    ext.extract_batch_device(d, kps, desc, cnt, stream=s)
    s.synchronize()
    assert torch.equal(cnt, ref[2])
    for b in range(B):
        n = int(cnt[b])
        assert torch.equal(kps[b, :n], ref[0][b, :n]) and torch.equal(desc[b, :n], ref[1][b, :n])
    assert lib.orb_stream_destroy(h) == 0
    assert lib.orb_stream_destroy(ctypes.c_void_p(0)) < 0


def test_release_stream_scratch_then_rerun():
    """1280x720 at nFeatures*2 (the reference's init extractor): ~1086 level-0 keypoints per
    frame, over k_match_init's LDS capacity, so every pair takes the large-capacity body and its
    per-stream scratch.  Release it, run again on the same stream: bit-exact both times."""
    import torch

    B, W, H = 3, 1280, 720
    frames = orb.synth_stream(W, H, stream=5, first=0, count=B)
    ext = orb.ORBextractor(5000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream())
        kps, desc, cnt = ext.extract_batch_device(d, stream=s)
    s.synchronize()
    n0 = [int((orb.keypoints_from_bytes(kps[b].cpu().numpy(), int(cnt[b]))["octave"] == 0).sum()) for b in range(B)]
    assert max(n0) > 1024, n0  # pairs over the LDS capacity: the large-capacity body
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    M = orb.ORBmatcher(0.9, True)
    outs = []
    for rep in range(2):
        m12, nm = M.search_for_initialization_batch_device(kps, desc, cnt, f1, f1 + 1, W, H, 100, stream=s)
        s.synchronize()
        outs.append((m12.cpu().numpy().copy(), nm.cpu().numpy().copy()))
        _check_pairs(kps, desc, cnt, m12, nm, W, H)
        assert orb.hip_lib().orb_match_release_stream_scratch(ctypes_stream(s)) == 0
    s.synchronize()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def ctypes_stream(s):
    import ctypes

    return ctypes.c_void_p(s.cuda_stream)
