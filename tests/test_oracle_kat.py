"""Known-answer tests that pin the oracle to values derived from the reference source
 and to the OpenCV-2.4 / glibc / libstdc++ behaviours it restates."""
import ctypes
import hashlib
import pathlib
import re

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import KEYPOINT_DTYPE, Oracle, _p, lib

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_umax_disc():
    # ORBextractor.cc:495-510
    _, _, _, um = Oracle(1000, 1.2, 8, 1, 20).level_info()
    assert um.tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert sum(2 * u + 1 for u in um[1:]) * 2 + 31 == 749  # pixels of the IC_Angle disc


@pytest.mark.parametrize("nf,expect", [
    (1000, [217, 181, 151, 126, 105, 87, 73, 60]),
    (2000, [434, 362, 302, 251, 209, 175, 145, 122]),
    (2500, [543, 452, 377, 314, 262, 218, 182, 152]),
])
def test_features_per_level(nf, expect):
    # ORBextractor.cc:476-487
    fpl, _, _, _ = Oracle(nf, 1.2, 8, 1, 20).level_info()
    assert fpl.tolist() == expect
    assert sum(expect) == nf


def test_scale_factors():
    # ORBextractor.cc:462-471: float accumulated through the double member scaleFactor
    _, sf, isf, _ = Oracle(1000, 1.2, 8, 1, 20).level_info()
    ref = [1.0, 1.2, 1.44, 1.728, 2.0736, 2.48832, 2.985984, 3.5831808]
    assert np.allclose(sf, ref, rtol=1e-6)
    acc = [np.float32(1.0)]
    for _ in range(7):
        acc.append(np.float32(np.float64(acc[-1]) * np.float64(np.float32(1.2))))
    assert sf.tobytes() == np.array(acc, np.float32).tobytes()
    inv = [np.float32(1.0)]
    f = np.float32(np.float32(1.0) / np.float64(np.float32(1.2)))
    for _ in range(7):
        inv.append(np.float32(inv[-1] * f))
    assert isf.tobytes() == np.array(inv, np.float32).tobytes()


def test_keypoint_size_per_level():
    # size = (int)(31 * mvScaleFactor[l]) (ORBextractor.cc:675)
    ora = Oracle(1000, 1.2, 8, 1, 20)
    k, _ = ora.extract(orb.synth_stream(640, 480, stream=1, count=1)[0])
    sizes = {int(o): float(s) for o, s in zip(k["octave"], k["size"])}
    assert [sizes[l] for l in range(8)] == [31, 37, 44, 53, 64, 77, 92, 111]
    assert (k["class_id"] == -1).all()


def test_pattern_table_hash_and_extent():
    # bit_pattern_31_ (ORBextractor.cc:197-455): SHA-256 prefix from SURVEY.md Appendix B
    text = (ROOT / "orbslam_jpminipc_amd" / "csrc" / "pattern31.inc").read_text()
    body = text[text.index("{") + 1: text.index("};")]
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(vals) == 1024
    assert hashlib.sha256(",".join(map(str, vals)).encode()).hexdigest().startswith("88df8ca875cc8db5")
    pts = np.array(vals).reshape(512, 2)
    assert pts.min() == -13 and pts.max() == 12
    r = np.sqrt((pts.astype(float) ** 2).sum(1)).max()
    assert 18.3 < r < 18.4  # rotated sample offsets stay within 18 px


def test_gaussian_taps():
    # getGaussianKernel(7, 2, CV_32F) * 256 -> [18,34,49,55,49,34,18], sum 257
    k = np.zeros(7, np.int32)
    lib().oracle_gaussian_taps(_p(k))
    assert k.tolist() == [18, 34, 49, 55, 49, 34, 18]
    assert k.sum() == 257


def test_blur_of_flat_image_brightens():
    # the 257/256 fixed-point gain: a flat 128 level blurs to 129 everywhere
    w, h = 40, 30
    padded = np.full((h + 32, w + 32), 128, np.uint8)
    out = np.zeros((h, w), np.uint8)
    lib().oracle_blur_padded(_p(padded), w, h, _p(out))
    assert (out == 129).all()
    padded[:] = 255
    lib().oracle_blur_padded(_p(padded), w, h, _p(out))
    assert (out == 255).all()  # saturates


def test_blur_matches_direct_formula():
    # Independent statement of SURVEY.md A3 on random small levels: T = sum k_i k_j P; the
    # SSE2 body (x < 4*floor(w/4)) rounds T/65536 half-to-even, the scalar tail half-up.
    rng = np.random.default_rng(3)
    for _ in range(40):
        w, h = 7, 9  # x = 4, 5, 6 are tail columns
        padded = rng.integers(0, 256, size=(h + 32, w + 32)).astype(np.uint8)
        out = np.zeros((h, w), np.uint8)
        lib().oracle_blur_padded(_p(padded), w, h, _p(out))
        k = np.array([18, 34, 49, 55, 49, 34, 18])
        P = padded.astype(np.int64)
        for y in range(h):
            for x in range(w):
                T = int((k[:, None] * k[None, :] * P[16 + y - 3:16 + y + 4, 16 + x - 3:16 + x + 4]).sum())
                exp_up = (T + 32768) >> 16
                q, r = divmod(T, 65536)
                exp_even = q + (1 if (r > 32768 or (r == 32768 and q % 2 == 1)) else 0)
                assert out[y, x] == min(255, exp_up if x >= 4 else exp_even)


def test_resize_flat_and_linear():
    # fixed-point weights sum to 2048: a flat image resizes to itself
    lib_ = lib()
    src = np.full((100, 120), 77, np.uint8)
    dst = np.zeros((83, 100), np.uint8)
    assert lib_.oracle_resize(_p(src), 120, 120, 100, _p(dst), 100, 100, 83) == 0
    assert (dst == 77).all()
    # exact 2x steps take OpenCV's INTER_AREA branch: refused like an unsupported config
    dst2 = np.zeros((50, 60), np.uint8)
    assert lib_.oracle_resize(_p(src), 120, 120, 100, _p(dst2), 60, 60, 50) == -95


def test_descriptor_distance_kats():
    L = lib()
    a = np.zeros(32, np.uint8)
    b = np.full(32, 255, np.uint8)
    c = a.copy()
    c[7] = 16
    assert L.oracle_descriptor_distance(_p(a), _p(a)) == 0
    assert L.oracle_descriptor_distance(_p(a), _p(b)) == 256
    assert L.oracle_descriptor_distance(_p(a), _p(c)) == 1
    rng = np.random.default_rng(0)
    lib_hip = orb.hip_lib()
    for _ in range(200):
        x = rng.integers(0, 256, 32, dtype=np.uint8)
        y = rng.integers(0, 256, 32, dtype=np.uint8)
        ref = int(np.unpackbits(x ^ y).sum())
        assert L.oracle_descriptor_distance(_p(x), _p(y)) == ref
        assert lib_hip.orb_descriptor_distance(_p(x), _p(y)) == ref
        assert orb.ORBmatcher.DescriptorDistance(x, y) == ref


def test_rotation_bins_only_0_to_12():
    # round(rot * (1/30)) with rot in degrees: only bins 0..12 are reachable (a reference quirk
    # kept bit-for-bit: ORBmatcher.cc:606, 668-673)
    L = lib()
    bins = set()
    for a1 in np.linspace(0, 360, 181, dtype=np.float32):
        for a2 in np.linspace(0, 360, 37, dtype=np.float32):
            bins.add(L.oracle_rot_bin(float(a1), float(a2)))
    assert bins == set(range(13))
    assert L.oracle_rot_bin(10.0, 10.0) == 0
    assert L.oracle_rot_bin(0.0, 15.0) == 12  # -15 -> 345 -> round(11.5) = 12 (half away from zero)
    assert L.oracle_rot_bin(1e-6, 2e-6) in (0, 12)


def test_fast_cell_semantics():
    # cv::FAST on a cell-sized Mat: a single bright pixel on dark is a corner with score
    # S - 1 = 199; detection rows/cols are [3, n-3)
    img = np.zeros((20, 20), np.uint8)
    img[10, 10] = 200
    out = np.zeros((64, 3), np.int32)
    n = lib().oracle_fast(_p(img), 20, 20, 20, 20, _p(out), 64)
    assert n == 1 and tuple(out[0]) == (10, 10, 199)
    # a 3x3 blob: all 9 pixels are corners with equal scores -> strict 3x3 NMS keeps none
    blob = np.zeros((20, 20), np.uint8)
    blob[9:12, 9:12] = 200
    assert lib().oracle_fast(_p(blob), 20, 20, 20, 20, _p(out), 64) == 0
    # the same pixel at column 2 is outside the detection window
    img2 = np.zeros((20, 20), np.uint8)
    img2[10, 2] = 200
    n2 = lib().oracle_fast(_p(img2), 20, 20, 20, 20, _p(out), 64)
    assert n2 == 0
    # flat image: nothing
    assert lib().oracle_fast(_p(np.full((20, 20), 90, np.uint8)), 20, 20, 20, 20, _p(out), 64) == 0


def test_extract_output_contract():
    ora = Oracle(1000, 1.2, 8, 1, 20)
    k, d = ora.extract(orb.synth_stream(640, 480, stream=2, count=1)[0])
    assert len(k) == 1000 and d.shape == (1000, 32)
    # level-major order; per level exactly the quota when the frame is textured enough
    assert (np.diff(k["octave"]) >= 0).all()
    assert np.bincount(k["octave"]).tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert ((k["angle"] >= 0) & (k["angle"] <= 360)).all()
    # keypoints keep the 16 px (scaled) border
    for l, s in enumerate([1, 1.2, 1.44, 1.728, 2.0736, 2.48832, 2.985984, 3.5831808]):
        kl = k[k["octave"] == l]
        assert kl["x"].min() >= 16 * s - 1e-3 and kl["y"].min() >= 16 * s - 1e-3
    # flat frame: no keypoints
    k0, d0 = ora.extract(np.full((480, 640), 128, np.uint8))
    assert len(k0) == 0
