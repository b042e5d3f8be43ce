"""The FAST strength arithmetic of `fast_strength_packed` (orb_hip.hip): contrasts as exact f16
denormals (a byte b loaded into a register is the binary16 bit pattern b = b * 2^-24), arcs of
9 as three windows of 3 (the kernel's v_pk_minimum3_f16), the best arc by maximum, and the
result read back as the int16 view of its bits.  Emulated here in numpy float16 (IEEE
binary16 with gradual underflow, the same as the hardware with f16 denormals enabled, which
the kernels' code objects declare: .amdhsa_float_denorm_mode_16_64 3) and checked (1) to stay
exact: every intermediate equals the integer value times 2^-24; (2) to give S = 1 + cornerScore
of cv::FAST, against the oracle's FAST (ORBextractor.cc:602 `FAST(..., true)`) on
7x7 patches: a corner at threshold t iff S > t, response S - 1."""
import ctypes

import numpy as np

from oracle_lib import lib

# circle order of the kernel's off[16] table: (dy, dx)
CIRCLE = [(3, 0), (3, 1), (2, 2), (1, 3), (0, 3), (-1, 3), (-2, 2), (-3, 1),
          (-3, 0), (-3, -1), (-2, -2), (-1, -3), (0, -3), (1, -3), (2, -2), (3, -1)]


def _arcs(d):
    """max over the 16 arcs of 9 of the arc minimum, by windows of 3 (d: (N, 16))."""
    m3 = np.minimum(np.minimum(d, np.roll(d, -1, axis=1)), np.roll(d, -2, axis=1))
    w9 = np.minimum(np.minimum(m3, np.roll(m3, -3, axis=1)), np.roll(m3, -6, axis=1))
    return w9.max(axis=1), m3, w9


def _den(b):
    """bytes -> the binary16 values with those bit patterns (denormals b * 2^-24)"""
    return b.astype(np.uint16).view(np.float16)


def strength_f16(v, c):
    V = _den(v)[:, None]
    C = _den(c)
    out, inter = [], []
    for d in (V - C, C - V):  # (v - c, c - v): the kernel's two f16 lanes
        best, m3, w9 = _arcs(d)
        out.append(best)
        inter += [d, m3, w9, best]
    # the kernel's read-back: int16 view of each lane's bits (negatives and -0 come out < 0),
    # the larger of the two lanes
    S = np.maximum(out[0].view(np.int16), out[1].view(np.int16)).astype(np.int32)
    return S, inter


def strength_int(v, c):
    vi = v.astype(np.int32)[:, None]
    ci = c.astype(np.int32)
    out, inter = [], []
    for d in (vi - ci, ci - vi):
        best, m3, w9 = _arcs(d)
        out.append(best)
        inter += [d, m3, w9, best]
    return np.maximum(out[0], out[1]), inter


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 256, n).astype(np.uint8)
    c = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    # corner-like rings: a bright or dark arc of 9..16 around v, the rest random
    k = rng.integers(0, 16, n)
    ln = rng.integers(9, 17, n)
    sign = rng.choice([-1, 1], n)
    for i in range(n // 2):
        for j in range(ln[i]):
            c[i, (k[i] + j) % 16] = np.clip(int(v[i]) + sign[i] * rng.integers(1, 200), 0, 255)
    # extremes
    v[:256] = np.arange(256)
    c[:128] = 0
    c[128:256] = 255
    return v, c


def test_f16_strength_is_exact():
    v, c = _cases(20000, 1)
    sf, inf = strength_f16(v, c)
    si, ini = strength_int(v, c)
    for a, b in zip(inf, ini):
        assert np.array_equal((a.astype(np.float64) * 2.0 ** 24), b), "an f16 intermediate is not exact"
    # S > 0 exactly; S <= 0 reads back <= 0 (no corner at any threshold >= 0)
    assert np.array_equal(np.where(si > 0, sf, 0), np.where(si > 0, si, 0))
    assert (sf[si <= 0] <= 0).all()
    assert si.min() >= -255 and si.max() <= 255


def test_f16_strength_is_cornerscore_plus_one():
    v, c = _cases(3000, 2)
    S = strength_f16(v, c)[0]
    rng = np.random.default_rng(3)
    L = lib()
    out = np.zeros(3 * 4, np.int32)
    n_corner = 0
    for i in range(len(v)):
        p = np.zeros((7, 7), np.uint8)
        p[3, 3] = v[i]
        for k, (dy, dx) in enumerate(CIRCLE):
            p[3 + dy, 3 + dx] = c[i, k]
        t = int(rng.integers(1, 80))
        n = L.oracle_fast(p.ctypes.data_as(ctypes.c_void_p), 7, 7, 7, t,
                          out.ctypes.data_as(ctypes.c_void_p), 4)
        assert n == (1 if S[i] > t else 0), f"case {i}: S {S[i]}, t {t}, oracle corners {n}"
        if n:
            n_corner += 1
            assert (out[0], out[1]) == (3, 3) and out[2] == S[i] - 1, f"case {i}: response {out[2]} vs S-1 {S[i] - 1}"
    assert n_corner > 300  # the corner-like half is exercised
