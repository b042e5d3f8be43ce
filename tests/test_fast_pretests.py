"""CPU proofs of the FAST pre-tests the kernels use before the exact strength (orb_hip.hip
compass_half / compass8_half; reference cv::FAST behind ORBextractor.cc:607 and 613).

* compass_half: per 16-bit lane, M = min(max(q0, q8), max(q4, q12)), m = max(min(q0, q8),
  min(q4, q12)); the pixel passes <=> t - max(M - v, v - m) < 0.  Restated here on i16 lanes
  and compared with the four-point definition (bright: a bright point in both pairs {0, 8} and
  {4, 12}; dark likewise) over all thresholds.
* Both pre-tests are necessary conditions of a FAST-9 corner: every pixel whose exact score
  (the oracle's 9-arc definition) exceeds t passes the four-point and the eight-point test.
"""
import numpy as np

# circle offsets (dy, dx) in cv::FAST order, index 0 = (3, 0) (orb_hip.hip fast_strength_packed)
CIRCLE = [(3, 0), (3, 1), (2, 2), (1, 3), (0, 3), (-1, 3), (-2, 2), (-3, 1),
          (-3, 0), (-3, -1), (-2, -2), (-1, -3), (0, -3), (1, -3), (2, -2), (3, -1)]


def score_gt(v, c, t):
    """Corner at t <=> 9 consecutive circle points all > v + t or all < v - t."""
    bright = c > v[:, None] + t
    dark = c < v[:, None] - t
    out = np.zeros(len(v), bool)
    for k in range(16):
        idx = [(k + i) % 16 for i in range(9)]
        out |= bright[:, idx].all(1) | dark[:, idx].all(1)
    return out


def compass_half(v, q0, q4, q8, q12, t):
    """The kernel's lane arithmetic (values 0..255 in i16 lanes)."""
    M = np.minimum(np.maximum(q0, q8), np.maximum(q4, q12)).astype(np.int16)
    m = np.maximum(np.minimum(q0, q8), np.minimum(q4, q12)).astype(np.int16)
    X = np.maximum(M - v, v - m).astype(np.int16)
    return (np.int16(t) - X) < 0


def compass8_half(v, c, t):
    q = [c[:, k].astype(np.int16) for k in range(16)]
    pairs = [(0, 8), (4, 12), (2, 10), (6, 14)]
    M = np.minimum.reduce([np.maximum(q[a], q[b]) for a, b in pairs])
    m = np.maximum.reduce([np.minimum(q[a], q[b]) for a, b in pairs])
    X = np.maximum(M - v, v - m).astype(np.int16)
    return (np.int16(t) - X) < 0


def test_compass_half_equals_four_point_definition():
    rng = np.random.default_rng(5)
    n = 2048
    for t in range(0, 256, 3):
        v = rng.integers(0, 256, n).astype(np.int16)
        q = rng.integers(0, 256, (4, n)).astype(np.int16)
        got = compass_half(v, q[0], q[1], q[2], q[3], t)
        T = t
        br = ((q[0] > v + T) | (q[2] > v + T)) & ((q[1] > v + T) | (q[3] > v + T))
        dk = ((q[0] < v - T) | (q[2] < v - T)) & ((q[1] < v - T) | (q[3] < v - T))
        assert np.array_equal(got, br | dk), t


def test_pretests_are_necessary_for_corners():
    rng = np.random.default_rng(9)
    n = 20000
    for t in (0, 7, 20, 40):
        v = rng.integers(0, 256, n).astype(np.int16)
        # circles biased towards corners: a random 9..16 arc pushed bright or dark
        c = rng.integers(0, 256, (n, 16)).astype(np.int16)
        start = rng.integers(0, 16, n)
        length = rng.integers(9, 17, n)
        sign = rng.choice([-1, 1], n)
        arc = ((np.arange(16)[None, :] - start[:, None]) % 16) < length[:, None]
        pushed = np.clip(v[:, None].astype(int) + sign[:, None] * (t + 1 + rng.integers(0, 30, (n, 16))), 0, 255)
        c = np.where(arc, pushed, c).astype(np.int16)
        corner = score_gt(v, c, t)
        assert corner.sum() > n // 4
        four = compass_half(v, c[:, 0], c[:, 4], c[:, 8], c[:, 12], t)
        eight = compass8_half(v, c, t)
        assert not (corner & ~four).any(), t
        assert not (corner & ~eight).any(), t
        # the eight-point test is the stronger filter
        assert not (eight & ~four).any(), t
