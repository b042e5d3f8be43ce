"""k_pyr_stream (the whole pyramid of a frame in one streaming pass) vs the per-level launches
(k_pyr0 + k_pyr_resize + k_pyr_resize_tail) and vs the oracle's ComputePyramid
(ORBextractor.cc:781-822): every padded level of every frame byte-identical, and identical
keypoints / descriptors, at the BASELINE sizes, odd sizes and unaligned input rows."""
import ctypes

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu


def _levels(ext, b):
    lib = orb.hip_lib()
    out = []
    for l in range(ext.nlevels):
        w, h = ctypes.c_int(), ctypes.c_int()
        assert lib.orb_debug_level_image(ext._h, b, l, None, ctypes.byref(w), ctypes.byref(h)) == 0
        g = np.empty((h.value + 32, w.value + 32), np.uint8)
        assert lib.orb_debug_level_image(ext._h, b, l, g.ctypes.data_as(ctypes.c_void_p), None, None) == 0
        out.append(g)
    return out


def _run(ext, d, mode):
    import torch

    lib = orb.hip_lib()
    assert lib.orb_debug_set_pyramid_path(ext._h, mode) == 0
    kps, desc, counts = ext.extract_batch_device(d)
    torch.cuda.synchronize()
    B = d.shape[0]
    lv = [_levels(ext, b) for b in range(B)]
    return kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy(), lv


def _plan(ext):
    k0, nr, lds = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    ok = orb.hip_lib().orb_debug_pyramid_plan(ext._h, ctypes.byref(k0), ctypes.byref(nr), ctypes.byref(lds))
    return ok, k0.value, nr.value, lds.value


@pytest.mark.parametrize("W,H,nf,nl", [(640, 480, 1000, 8), (1241, 376, 2000, 8), (1280, 720, 2500, 8),
                                       (641, 479, 1000, 8), (320, 240, 1000, 8), (161, 121, 300, 4),
                                       (752, 480, 1000, 8)])
def test_stream_pyramid_equals_per_level(W, H, nf, nl):
    import torch

    B = 3
    frames = orb.synth_stream(W, H, stream=7, first=0, count=B)
    ext = orb.ORBextractor(nf, 1.2, nl, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    ref = _run(ext, d, 1)
    ok, k0, nr, lds = _plan(ext)
    assert ok == 1, "every BASELINE-like size has a stream plan"
    assert 1 <= k0 <= 32 and nr >= (H + k0 - 1) // k0 and 0 < lds <= 76 * 1024
    got = _run(ext, d, 2)
    for b in range(B):
        for l in range(nl):
            assert np.array_equal(got[3][b][l], ref[3][b][l]), \
                f"frame {b} level {l} differs at {np.argwhere(got[3][b][l] != ref[3][b][l])[:5]}"
    assert np.array_equal(got[2], ref[2])
    for b in range(B):
        n = ref[2][b]
        assert got[0][b, :n].tobytes() == ref[0][b, :n].tobytes()
        assert got[1][b, :n].tobytes() == ref[1][b, :n].tobytes()
    # and the oracle's pyramid (frame 0)
    ora = Oracle(nf, 1.2, nl, 1, 20)
    ko, do = ora.extract(frames[0])
    for l in range(nl):
        assert np.array_equal(got[3][0][l], ora.level_image(l)), f"level {l} differs from the oracle"
    assert got[0][0, :len(ko)].tobytes() == ko.tobytes() and got[2][0] == len(ko)
    orb.hip_lib().orb_debug_set_pyramid_path(ext._h, 0)


@pytest.mark.parametrize("offset,extra", [(1, 3), (4, 12), (16, 16)])
def test_stream_pyramid_unaligned_rows(offset, extra):
    """Input rows at byte / dword / 16-byte alignment (k_pyr_stream's three load widths)."""
    import torch

    B, W, H = 2, 640, 480
    frames = orb.synth_stream(W, H, stream=9, first=0, count=B)
    stride = W + extra
    buf = torch.zeros(offset + B * H * stride + 64, dtype=torch.uint8)
    view = buf[offset:offset + B * H * stride].view(B, H, stride)
    view[:, :, :W] = torch.from_numpy(frames)
    d_buf = buf.cuda()
    d = d_buf[offset:offset + B * H * stride].view(B, H, stride)[:, :, :W]
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    ref = _run(ext, d, 1)
    got = _run(ext, d, 2)
    for b in range(B):
        for l in range(8):
            assert np.array_equal(got[3][b][l], ref[3][b][l]), f"frame {b} level {l}"
        n = ref[2][b]
        assert got[2][b] == n and got[0][b, :n].tobytes() == ref[0][b, :n].tobytes()


def test_stream_pyramid_default_large_batch_sampled():
    """The automatic path at B = 256 (k_pyr_stream) against the per-level path on the same
    batch: all 256 frames' keypoints and descriptors, and the pyramid of a few frames."""
    import torch

    B, W, H = 256, 640, 480
    frames = orb.synth_stream(W, H, stream=4, first=100, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    lib = orb.hip_lib()
    lib.orb_debug_set_pyramid_path(ext._h, 1)
    k1, d1, c1 = [t.cpu().numpy() for t in ext.extract_batch_device(d)]
    lv1 = {b: _levels(ext, b) for b in (0, 77, 255)}
    lib.orb_debug_set_pyramid_path(ext._h, 0)
    k0, d0, c0 = [t.cpu().numpy() for t in ext.extract_batch_device(d)]
    torch.cuda.synchronize()
    assert np.array_equal(c0, c1)
    for b in range(B):
        n = c1[b]
        assert k0[b, :n].tobytes() == k1[b, :n].tobytes(), f"frame {b}"
        assert d0[b, :n].tobytes() == d1[b, :n].tobytes(), f"frame {b}"
    for b, ref in lv1.items():
        got = _levels(ext, b)
        for l in range(8):
            assert np.array_equal(got[l], ref[l]), f"frame {b} level {l}"



@pytest.mark.parametrize("W,H,nf,sf,nl", [(1920, 1080, 3000, 1.2, 8), (1024, 768, 1500, 1.5, 5),
                                          (800, 600, 1200, 1.25, 7)])
def test_stream_pyramid_other_geometries(W, H, nf, sf, nl):
    """Wider frames (smaller rounds) and other scale factors (other tap tables): the stream
    plan, when the geometry has one, gives the per-level pyramid byte for byte."""
    import torch

    B = 2
    frames = orb.synth_stream(W, H, stream=5, first=0, count=B)
    ext = orb.ORBextractor(nf, sf, nl, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    ref = _run(ext, d, 1)
    ok, k0, nr, lds = _plan(ext)
    if not ok:
        pytest.skip(f"no stream plan for {W}x{H} (per-level path only)")
    got = _run(ext, d, 2)
    for b in range(B):
        for l in range(nl):
            assert np.array_equal(got[3][b][l], ref[3][b][l]), f"frame {b} level {l}"
        n = ref[2][b]
        assert got[2][b] == n and got[0][b, :n].tobytes() == ref[0][b, :n].tobytes()
        assert got[1][b, :n].tobytes() == ref[1][b, :n].tobytes()
    orb.hip_lib().orb_debug_set_pyramid_path(ext._h, 0)
