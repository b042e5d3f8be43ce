"""CPU checks of the integer / float identities k_orient_desc relies on (orb_hip.hip):

* the blur row pass as an i8 x i8 -> i32 matrix product (v_mfma_i32_16x16x64_i8): window bytes
  recentred by p ^ 0x80 (= p - 128 as i8), the banded 7-tap matrix B[k][n] = tap[k - n], and
  columns 61..63 carrying (127, 127, 11) in A and (127, 127, 58) in B, so that
  A x B = sum_j tap[j] * p[n + j] exactly for every output column the column pass reads
  (n <= 54); the B table is built exactly as upload_pattern() builds c_rowB;
* cvRound of the rBRIEF sample offsets as the low mantissa bits of v + (1.5 * 2^23 + 18).

Both are exact-arithmetic identities; the GPU parity tests check the kernel itself.
"""
import numpy as np

TAP = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)  # GaussianBlur 7x7 sigma 2, fixed point


def rowb_matrix():
    """B[k][n] for window columns k, n in 0..63 (the c_rowB fragments, before the lane split)."""
    B = np.zeros((64, 64), np.int64)
    for k in range(64):
        for n in range(64):
            if 0 <= k - n <= 6:
                B[k, n] = TAP[k - n]
            if k >= 61:
                B[k, n] = 58 if k == 63 else 127
    assert B.min() >= -128 and B.max() <= 127  # i8 operand
    return B


def test_rowpass_mfma_bias_exact():
    rng = np.random.default_rng(7)
    B = rowb_matrix()
    for trial in range(200):
        if trial == 0:
            win = np.zeros((44, 64), np.uint8)
        elif trial == 1:
            win = np.full((44, 64), 255, np.uint8)
        else:
            win = rng.integers(0, 256, (44, 64), dtype=np.uint8)
        A = (win ^ 0x80).view(np.int8).astype(np.int64)  # p - 128
        A[:, 61:64] = (127, 127, 11)
        assert A.min() >= -128 and A.max() <= 127
        H = A @ B
        direct = np.stack([win[:, n:n + 7].astype(np.int64) @ TAP for n in range(55)], axis=1)
        assert np.array_equal(H[:, :55], direct)
        assert H[:, :55].max() <= 65535 and H[:, :55].min() >= 0  # one u16 per sum


def test_rowpass_band_never_reaches_bias_columns():
    # sum column hc (0..39) of a keypoint at window offset o0 (0..15) reads window columns
    # o0 + hc .. o0 + hc + 6 <= 60
    assert max(o0 + hc + 6 for o0 in range(16) for hc in range(40)) == 60


def test_magic_cvround():
    rng = np.random.default_rng(3)
    v = np.concatenate([
        rng.uniform(-20, 20, 200000).astype(np.float32),
        (np.arange(-40, 41) / 2).astype(np.float32),  # exact halves: ties to even
        np.nextafter(np.float32(0.5), np.float32(0)) * np.array([1, -1], np.float32),
        np.array([-0.0, 0.0], np.float32),
    ])
    s = (v + np.float32(12582930.0)).astype(np.float32)
    got = s.view(np.uint32).astype(np.int64) - 0x4B400012
    assert np.array_equal(got, np.rint(v).astype(np.int64))
