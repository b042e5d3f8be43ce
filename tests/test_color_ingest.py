"""Tracking::GrabImage's colour conversion fused into the extractor's level-0 pass (reference
src/Tracking.cc:202-207; OpenCV 2.4 RGB2Gray<uchar>): oracle known answers and a numpy
restatement on the CPU; GPU extraction from colour frames bit-exact against the oracle's gray
conversion followed by the oracle extractor."""
import ctypes

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle, _p, lib


def rgb_to_gray(img, rgb):
    L = lib()
    L.oracle_rgb_to_gray.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    img = np.ascontiguousarray(img, np.uint8)
    h, w, cn = img.shape
    out = np.empty((h, w), np.uint8)
    assert L.oracle_rgb_to_gray(_p(img), w, h, w * cn, cn, int(rgb), _p(out)) == 0
    return out


def color_frame(gray, seed, cn=3):
    rng = np.random.default_rng(seed)
    g = gray.astype(np.int32)
    r = np.clip(g + rng.integers(-20, 21, g.shape), 0, 255)
    b = np.clip(255 - g + rng.integers(-10, 11, g.shape), 0, 255)
    ch = [r, g, b] + ([np.full(g.shape, 9)] if cn == 4 else [])
    return np.stack(ch, axis=2).astype(np.uint8)


def test_oracle_known_answers():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [77, 77, 77]]], np.uint8)
    assert rgb_to_gray(px, True).tolist() == [[76, 150, 29, 255, 77]]  # OpenCV's published values
    assert rgb_to_gray(px, False).tolist() == [[29, 150, 76, 255, 77]]


@pytest.mark.parametrize("rgb", [True, False])
def test_oracle_matches_numpy(rgb):
    img = np.random.default_rng(1).integers(0, 256, size=(37, 53, 4), dtype=np.uint8)
    c = (4899, 9617, 1868) if rgb else (1868, 9617, 4899)
    p = img.astype(np.int64)
    ref = (c[0] * p[..., 0] + c[1] * p[..., 1] + c[2] * p[..., 2] + 8192) >> 14
    assert np.array_equal(rgb_to_gray(img, rgb), ref.astype(np.uint8))


def test_colour_entry_point_rejects_gray_input():
    # validated before any library call (an extractor handle itself needs a device)
    with pytest.raises(TypeError):
        orb.ORBextractor.extract_color(object.__new__(orb.ORBextractor), np.zeros((4, 4), np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("rgb,cn", [(True, 3), (False, 3), (True, 4)])
def test_gpu_colour_extraction(rgb, cn):
    import torch

    W, H = 640, 480
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=3)
    ora = Oracle(1000, 1.2, 8, 1, 20)
    cols = [color_frame(g, i, cn) for i, g in enumerate(orb.synth_stream(W, H, stream=70, first=0, count=3))]
    for c in cols:
        kg, dg = ext.extract_color(c, rgb=rgb)
        ko, do = ora.extract(rgb_to_gray(c, rgb))
        assert kg.tobytes() == ko.tobytes() and dg.tobytes() == do.tobytes()
    k, de, n = ext.extract_batch_device_color(torch.from_numpy(np.stack(cols)).cuda(), rgb=rgb)
    torch.cuda.synchronize()
    k, de, n = k.cpu().numpy(), de.cpu().numpy(), n.cpu().numpy()
    for b, c in enumerate(cols):
        ko, do = ora.extract(rgb_to_gray(c, rgb))
        assert n[b] == len(ko)
        assert k[b, :n[b]].tobytes() == ko.tobytes() and de[b, :n[b]].tobytes() == do.tobytes()
