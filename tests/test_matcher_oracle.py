"""The oracle's matcher vs a second, pure-Python restatement of the reference (small cases).

Follows ORBmatcher.cc:598-713 (SearchForInitialization), 155-284 / 715-850 (SearchByBoW),
1748-1789 (ComputeThreeMaxima) and Frame.cc:200-277 (grid + GetFeaturesInArea) line by
line in plain Python with numpy float32 scalars, so the C++ oracle is checked by an
independent reading on inputs that exercise stealing, stale histogram entries and ties.
"""
import ctypes

import numpy as np
import pytest

from oracle_lib import KEYPOINT_DTYPE, _Bounds, _p, lib

F32 = np.float32
INT_MAX = 2**31 - 1


def hamming(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


class PyFrame:
    def __init__(self, kps, desc, W, H):
        self.k, self.d = kps, desc
        self.minX, self.maxX, self.minY, self.maxY = 0, W, 0, H
        self.invW = F32(64) / F32(W)
        self.invH = F32(48) / F32(H)
        self.grid = {}
        for i, kp in enumerate(kps):
            # std::round (half away from zero) of a non-negative float32 product
            px = int(np.floor(np.float64(F32(kp["x"] - F32(self.minX)) * self.invW) + 0.5))
            py = int(np.floor(np.float64(F32(kp["y"] - F32(self.minY)) * self.invH) + 0.5))
            if 0 <= px < 64 and 0 <= py < 48:
                self.grid.setdefault((px, py), []).append(i)

    def area(self, x, y, r, minL, maxL):
        x, y, r = F32(x), F32(y), F32(r)
        out = []
        nminx = max(0, int(np.floor(F32(F32(x - F32(self.minX)) - r) * self.invW)))
        if nminx >= 64:
            return out
        nmaxx = min(63, int(np.ceil(F32(F32(x - F32(self.minX)) + r) * self.invW)))
        if nmaxx < 0:
            return out
        nminy = max(0, int(np.floor(F32(F32(y - F32(self.minY)) - r) * self.invH)))
        if nminy >= 48:
            return out
        nmaxy = min(47, int(np.ceil(F32(F32(y - F32(self.minY)) + r) * self.invH)))
        if nmaxy < 0:
            return out
        check = not (minL == -1 and maxL == -1)
        same = check and minL == maxL
        for ix in range(nminx, nmaxx + 1):
            for iy in range(nminy, nmaxy + 1):
                for j in self.grid.get((ix, iy), []):
                    kp = self.k[j]
                    if check and not same and (kp["octave"] < minL or kp["octave"] > maxL):
                        continue
                    if same and kp["octave"] != minL:
                        continue
                    if abs(F32(kp["x"] - x)) > r or abs(F32(kp["y"] - y)) > r:
                        continue
                    out.append(j)
        return out


def three_maxima(hist):
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, h in enumerate(hist):
        s = len(h)
        if s > max1:
            max3, max2, max1 = max2, max1, s
            i3, i2, i1 = i2, i1, i
        elif s > max2:
            max3, max2 = max2, s
            i3, i2 = i2, i
        elif s > max3:
            max3, i3 = s, i
    if max2 < F32(0.1) * F32(max1):
        i2 = i3 = -1
    elif max3 < F32(0.1) * F32(max1):
        i3 = -1
    return i1, i2, i3


def rot_bin(a1, a2):
    rot = F32(F32(a1) - F32(a2))
    if rot < 0.0:
        rot = F32(rot + F32(360.0))
    v = np.float64(F32(rot * F32(F32(1.0) / F32(30))))
    b = int(np.floor(v + 0.5))  # std::round of a non-negative value
    return 0 if b == 30 else b


def py_search_for_initialization(F1, F2, prev, nnratio, check_ori, window):
    n1 = len(F1.k)
    m12 = [-1] * n1
    hist = [[] for _ in range(30)]
    md = [INT_MAX] * len(F2.k)
    m21 = [-1] * len(F2.k)
    nm = 0
    for i1 in range(n1):
        lvl = int(F1.k[i1]["octave"])
        if lvl > 0:
            continue
        cands = F2.area(prev[i1, 0], prev[i1, 1], window, lvl, lvl)
        if not cands:
            continue
        best = best2 = INT_MAX
        bidx = -1
        for i2 in cands:
            dist = hamming(F1.d[i1], F2.d[i2])
            if md[i2] <= dist:
                continue
            if dist < best:
                best2, best, bidx = best, dist, i2
            elif dist < best2:
                best2 = dist
        if best <= 50 and F32(best) < F32(F32(best2) * F32(nnratio)):
            if m21[bidx] >= 0:
                m12[m21[bidx]] = -1
                nm -= 1
            m12[i1] = bidx
            m21[bidx] = i1
            md[bidx] = best
            nm += 1
            if check_ori:
                hist[rot_bin(F1.k[i1]["angle"], F2.k[bidx]["angle"])].append(i1)
    if check_ori:
        keep = three_maxima(hist)
        for i in range(30):
            if i in keep:
                continue
            for i1 in hist[i]:
                if m12[i1] >= 0:
                    m12[i1] = -1
                    nm -= 1
    for i1 in range(n1):
        if m12[i1] >= 0:
            prev[i1] = (F2.k[m12[i1]]["x"], F2.k[m12[i1]]["y"])
    return nm, np.array(m12, np.int32)


def make_pair(rng, n1, n2, W=640, H=480, flips=(0, 30), noise_frac=0.4):
    """F2 = F1 moved a little with descriptor bit flips; extra random keypoints; many ties."""
    k1 = np.zeros(n1, KEYPOINT_DTYPE)
    k1["x"] = rng.integers(16, W - 16, n1)
    k1["y"] = rng.integers(16, H - 16, n1)
    k1["octave"] = rng.choice([0, 0, 0, 1, 2], n1)
    k1["angle"] = rng.uniform(0, 360, n1).astype(np.float32)
    k1["response"] = rng.integers(20, 60, n1)
    k1["class_id"] = -1
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    k2 = np.zeros(n2, KEYPOINT_DTYPE)
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    m = min(n1, n2)
    k2[:m] = k1[:m]
    k2["x"][:m] += rng.integers(-5, 6, m)
    k2["y"][:m] += rng.integers(-5, 6, m)
    k2["angle"][:m] = (k1["angle"][:m] + rng.normal(0, 8, m).astype(np.float32)) % 360
    for j in range(m):
        if rng.random() < noise_frac:
            continue
        nf = int(rng.integers(*flips))
        d2[j] = d1[j]
        for b in rng.choice(256, nf, replace=False):
            d2[j, b // 8] ^= 1 << (b % 8)
    if n2 > m:
        k2["x"][m:] = rng.integers(16, W - 16, n2 - m)
        k2["y"][m:] = rng.integers(16, H - 16, n2 - m)
        k2["octave"][m:] = rng.choice([0, 1], n2 - m)
        k2["angle"][m:] = rng.uniform(0, 360, n2 - m)
    # duplicate some F2 descriptors to force distance ties and stealing
    for j in rng.choice(n2, n2 // 6, replace=False):
        d2[j] = d2[rng.integers(0, n2)]
    perm = rng.permutation(n2)
    return k1, d1, k2[perm].copy(), d2[perm].copy()


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("nnratio,check_ori,window", [(0.9, True, 100), (0.6, True, 30), (0.75, False, 60)])
def test_search_for_initialization_vs_python(seed, nnratio, check_ori, window):
    rng = np.random.default_rng(seed)
    k1, d1, k2, d2 = make_pair(rng, int(rng.integers(40, 160)), int(rng.integers(40, 160)))
    F1, F2 = PyFrame(k1, d1, 640, 480), PyFrame(k2, d2, 640, 480)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    prev_o = prev.copy()
    nm_py, m12_py = py_search_for_initialization(F1, F2, prev, nnratio, check_ori, window)
    L = lib()
    m12 = np.full(len(k1), -1, np.int32)
    n = ctypes.c_int()
    assert L.oracle_search_for_initialization(_p(k1), _p(d1), len(k1), _p(k2), _p(d2), len(k2),
                                              _Bounds(0, 640, 0, 480), nnratio, int(check_ori), window,
                                              _p(prev_o), _p(m12), ctypes.byref(n)) == 0
    assert n.value == nm_py
    assert np.array_equal(m12, m12_py)
    assert prev_o.tobytes() == prev.tobytes()


def test_features_in_area_vs_python():
    rng = np.random.default_rng(11)
    k1, d1, _, _ = make_pair(rng, 300, 10)
    F = PyFrame(k1, d1, 640, 480)
    L = lib()
    out = np.zeros(400, np.int32)
    for _ in range(200):
        x, y = rng.uniform(-50, 700), rng.uniform(-50, 530)
        r = float(rng.choice([5, 10, 50, 100, 200]))
        lo, hi = [(-1, -1), (0, 0), (0, 1), (1, 2)][int(rng.integers(0, 4))]
        n = L.oracle_features_in_area(_p(k1), len(k1), _Bounds(0, 640, 0, 480), float(x), float(y), r, lo, hi,
                                      _p(out), 400)
        assert out[:n].tolist() == F.area(x, y, r, lo, hi)


def _csr(rng, n, nodes_pool):
    """Random FeatureVector as CSR: node -> feature indices (each feature in one node)."""
    assign = rng.choice(nodes_pool, n)
    nodes = np.unique(assign).astype(np.uint32)
    off = [0]
    feat = []
    for nd in nodes:
        idx = np.nonzero(assign == nd)[0].tolist()
        feat += idx
        off.append(len(feat))
    return nodes, np.array(off, np.int32), np.array(feat, np.int32)


def py_bow_kf_f(kkf, dkf, valid, nkf, fk, fd, nf_, nnratio, check_ori):
    (n1, o1, f1), (n2, o2, f2) = nkf, nf_
    out = [-1] * len(fk)
    hist = [[] for _ in range(30)]
    nm = 0
    a = b = 0
    while a < len(n1) and b < len(n2):
        if n1[a] == n2[b]:
            for iKF in f1[o1[a]:o1[a + 1]]:
                if not valid[iKF]:
                    continue
                best = best2 = INT_MAX
                bidx = -1
                for iF in f2[o2[b]:o2[b + 1]]:
                    if out[iF] >= 0:
                        continue
                    dist = hamming(dkf[iKF], fd[iF])
                    if dist < best:
                        best2, best, bidx = best, dist, iF
                    elif dist < best2:
                        best2 = dist
                if best <= 50 and F32(best) < F32(F32(nnratio) * F32(best2)):
                    out[bidx] = int(iKF)
                    if check_ori:
                        hist[rot_bin(kkf[iKF]["angle"], fk[bidx]["angle"])].append(bidx)
                    nm += 1
            a += 1
            b += 1
        elif n1[a] < n2[b]:
            a = int(np.searchsorted(n1, n2[b]))
        else:
            b = int(np.searchsorted(n2, n1[a]))
    if check_ori:
        keep = three_maxima(hist)
        for i in range(30):
            if i in keep:
                continue
            for j in hist[i]:
                out[j] = -1
                nm -= 1
    return nm, np.array(out, np.int32)


@pytest.mark.parametrize("seed", range(6))
def test_search_by_bow_kf_f_vs_python(seed):
    rng = np.random.default_rng(100 + seed)
    k1, d1, k2, d2 = make_pair(rng, 120, 140, noise_frac=0.2)
    valid = (rng.random(len(k1)) < 0.8).astype(np.uint8)
    pool = np.arange(0, 400, 7)
    c1, c2 = _csr(rng, len(k1), pool), _csr(rng, len(k2), pool)
    nm_py, out_py = py_bow_kf_f(k1, d1, valid, c1, k2, d2, c2, 0.75, True)
    L = lib()
    out = np.zeros(len(k2), np.int32)
    n = ctypes.c_int()
    assert L.oracle_search_by_bow_kf_f(_p(k1), _p(d1), len(k1), _p(valid), _p(c1[0]), _p(c1[1]), _p(c1[2]),
                                       len(c1[0]), _p(k2), _p(d2), len(k2), _p(c2[0]), _p(c2[1]), _p(c2[2]),
                                       len(c2[0]), 0.75, 1, _p(out), ctypes.byref(n)) == 0
    assert n.value == nm_py
    assert np.array_equal(out, out_py)
