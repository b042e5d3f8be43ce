"""The oracle's matcher family (oracle/orb_oracle_match.cpp) vs a second, pure-Python reading
of the reference (small seeded scenes, CPU only).

Line-by-line restatements of ORBmatcher.cc (WindowSearch 409-516, SearchByProjection 49-125,
Fuse 1016-1265, SearchForTriangulation 852-1014 with CheckDistEpipolarLine 136-153),
Frame::isInFrustum (Frame.cc:137-198) and KeyFrame::GetFeaturesInArea (KeyFrame.cc:612-652)
in numpy float32 / float64 scalars.  Where g++ -O3 -march=native contracts an expression
into an FMA (scripts/contraction_check.sh), fma(a, b, c) is evaluated as the exact float64
a*b (a float32 product is exact in float64) plus c, rounded to float32.
"""
import math

import numpy as np
import pytest

import scenes as S
from oracle_lib import OracleMatcher
from orbslam_jpminipc_amd.views import View
from test_matcher_oracle import INT_MAX, F32, hamming, rot_bin, three_maxima

F64 = np.float64


def fma32(a, b, c):
    return F32(F64(F32(a)) * F64(F32(b)) + F64(F32(c)))


def std_round(v):  # half away from zero
    v = float(v)
    return int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))


class PyView:
    """Frame / KeyFrame grid and window queries (Frame.cc:200-277, KeyFrame.cc:612-657)."""

    def __init__(self, V: View):
        self.V, self.k, self.d = V, V.kps, V.desc
        self.minX, self.maxX, self.minY, self.maxY = V.bounds[0], V.bounds[1], V.bounds[2], V.bounds[3]
        self.invW = F32(F32(64) / F32(self.maxX - self.minX))
        self.invH = F32(F32(48) / F32(self.maxY - self.minY))
        self.grid = {}
        for i, kp in enumerate(self.k):
            px = std_round(F32(F32(kp["x"] - F32(self.minX)) * self.invW))
            py = std_round(F32(F32(kp["y"] - F32(self.minY)) * self.invH))
            if 0 <= px < 64 and 0 <= py < 48:
                self.grid.setdefault((px, py), []).append(i)

    def cells(self, x, y, r):
        nminx = max(0, int(np.floor(F32(F32(F32(x) - F32(self.minX)) - r) * self.invW)))
        if nminx >= 64:
            return None
        nmaxx = min(63, int(np.ceil(F32(F32(F32(x) - F32(self.minX)) + r) * self.invW)))
        if nmaxx < 0:
            return None
        nminy = max(0, int(np.floor(F32(F32(F32(y) - F32(self.minY)) - r) * self.invH)))
        if nminy >= 48:
            return None
        nmaxy = min(47, int(np.ceil(F32(F32(F32(y) - F32(self.minY)) + r) * self.invH)))
        if nmaxy < 0:
            return None
        return nminx, nmaxx, nminy, nmaxy

    def area(self, x, y, r, minL, maxL):
        x, y, r = F32(x), F32(y), F32(r)
        c = self.cells(x, y, r)
        out = []
        if c is None:
            return out
        check = not (minL == -1 and maxL == -1)
        same = check and minL == maxL
        for ix in range(c[0], c[1] + 1):
            for iy in range(c[2], c[3] + 1):
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

    def kf_area(self, x, y, r):
        x, y, r = F32(x), F32(y), F32(r)
        c = self.cells(x, y, r)
        out = []
        if c is None:
            return out
        for ix in range(c[0], c[1] + 1):
            for iy in range(c[2], c[3] + 1):
                for j in self.grid.get((ix, iy), []):
                    kp = self.k[j]
                    if abs(F32(kp["x"] - x)) <= r and abs(F32(kp["y"] - y)) <= r:
                        out.append(j)
        return out

    def in_image(self, u, v):
        return self.minX <= u < self.maxX and self.minY <= v < self.maxY

    def predict(self, ratio):
        sf = self.V.mvScaleFactors[:self.V.nlevels]
        n = 0
        while n < len(sf) and sf[n] < ratio:
            n += 1
        return min(n, self.V.nlevels - 1)


def gemm3_add(A, x, t):  # OpenCV 2.4 gemm small-size path (oracle/ocv_ops.h)
    A = np.asarray(A, F32).reshape(3, 3)
    out = np.zeros(3, F32)
    for i in range(3):
        ti = F32(F32(F32(A[i, 0] * x[0]) + F32(A[i, 1] * x[1])) + F32(A[i, 2] * x[2]))
        out[i] = F32(F64(ti) + F64(F32(t[i])))
    return out


def norm3(v):
    s = F64(0)
    for e in v:
        s = s + F64(e) * F64(e)
    return F64(np.sqrt(s))


def dot3(a, b):
    r = F64(0)
    for i in range(3):
        r = r + F64(a[i]) * F64(b[i])
    return r


def py_window_search(F1: View, usable1, F2: View, window, minL, maxL, nnratio, check_ori):
    P2 = PyView(F2)
    m21 = [-1] * F2.n
    hist = [[] for _ in range(30)]
    nm = 0
    for i1 in range(F1.n):
        if not usable1[i1]:
            continue
        kp1 = F1.kps[i1]
        l1 = int(kp1["octave"])
        if minL > 0 and l1 < minL:
            continue
        if maxL < INT_MAX and l1 > maxL:
            continue
        cands = P2.area(kp1["x"], kp1["y"], F32(window), l1, l1)
        if not cands:
            continue
        best = best2 = INT_MAX
        bidx = -1
        for i2 in cands:
            if m21[i2] >= 0:
                continue
            d = hamming(F1.desc[i1], F2.desc[i2])
            if d < best:
                best2, best, bidx = best, d, i2
            elif d < best2:
                best2 = d
        if F32(best) <= F32(F32(best2) * F32(nnratio)) and best <= 100:
            m21[bidx] = i1
            nm += 1
            hist[rot_bin(kp1["angle"], F2.kps[bidx]["angle"])].append(bidx)
    if check_ori:
        keep = three_maxima(hist)
        for i, h in enumerate(hist):
            if i in keep:
                continue
            for j in h:
                m21[j] = -1
                nm -= 1
    return nm, np.array(m21, np.int32)


def py_is_in_frustum(F: View, mps, lim):
    out = []
    for i in range(mps.n):
        P = mps.pos[i]
        Pc = gemm3_add(F.Rcw, P, F.tcw)
        if Pc[2] < 0.0:
            out.append((0, 0.0, 0.0, -1, 0.0))
            continue
        invz = F32(F64(1.0) / F64(Pc[2]))
        u = fma32(F32(F.fx * Pc[0]), invz, F.cx)
        v = fma32(F32(F.fy * Pc[1]), invz, F.cy)
        if u < F.bounds[0] or u > F.bounds[1] or v < F.bounds[2] or v > F.bounds[3]:
            out.append((0, 0.0, 0.0, -1, 0.0))
            continue
        PO = np.array([P[k] - F.Ow[k] for k in range(3)], F32)
        dist = F32(norm3(PO))
        if dist < mps.dmin[i] or dist > mps.dmax[i]:
            out.append((0, 0.0, 0.0, -1, 0.0))
            continue
        vc = F32(dot3(PO, mps.normal[i]) / F64(dist))
        if vc < F32(lim):
            out.append((0, 0.0, 0.0, -1, 0.0))
            continue
        ratio = F32(dist / mps.dmin[i])
        out.append((1, u, v, _predict(F, ratio), vc))
    return out


def _predict(V: View, ratio):
    sf = V.mvScaleFactors[:V.nlevels]
    n = 0
    while n < len(sf) and sf[n] < ratio:
        n += 1
    return min(n, V.nlevels - 1)


def py_sbp_local(F: View, taken, usable, px, py, lv, vc, mpdesc, th, nnratio):
    P = PyView(F)
    taken = list(taken)
    fm = [-1] * F.n
    nm = 0
    for i in range(len(px)):
        if not usable[i]:
            continue
        pred = int(lv[i])
        r = F32(2.5) if F64(vc[i]) > 0.998 else F32(4.0)
        if F32(th) != 1.0:
            r = F32(r * F32(th))
        cands = P.area(px[i], py[i], F32(r * F.mvScaleFactors[pred]), pred - 1, pred)
        if not cands:
            continue
        best = best2 = INT_MAX
        bl = bl2 = -1
        bidx = -1
        for idx in cands:
            if taken[idx]:
                continue
            d = hamming(mpdesc[i], F.desc[idx])
            if d < best:
                best2, best, bl2, bl, bidx = best, d, bl, int(F.kps[idx]["octave"]), idx
            elif d < best2:
                bl2, best2 = int(F.kps[idx]["octave"]), d
        if best <= 100:
            if bl == bl2 and F32(best) > F32(F32(nnratio) * F32(best2)):
                continue
            taken[bidx] = 1
            fm[bidx] = i
            nm += 1
    return nm, np.array(fm, np.int32)


def py_fuse(KF: View, pts, usable, th, scw):
    P = PyView(KF)
    out = [-1] * pts.n
    nf = 0
    for i in range(pts.n):
        if not usable[i]:
            continue
        p = pts.pos[i]
        X = gemm3_add(KF.Rcw, p, KF.tcw)
        if X[2] < 0.0:
            continue
        invz = F32(F64(1.0) / F64(X[2])) if scw else F32(F32(1.0) / X[2])
        x, y = F32(X[0] * invz), F32(X[1] * invz)
        u, v = fma32(KF.fx, x, KF.cx), fma32(KF.fy, y, KF.cy)
        if not P.in_image(u, v):
            continue
        PO = np.array([p[k] - KF.Ow[k] for k in range(3)], F32)
        d3 = F32(norm3(PO))
        if d3 < pts.dmin[i] or d3 > pts.dmax[i]:
            continue
        if dot3(PO, pts.normal[i]) < 0.5 * F64(d3):
            continue
        pred = P.predict(F32(d3 / pts.dmin[i]))
        cands = P.kf_area(u, v, F32(F32(th) * KF.mvScaleFactors[pred]))
        best, bidx = INT_MAX, -1
        for idx in cands:
            lvl = int(KF.kps[idx]["octave"])
            if lvl < pred - 1 or lvl > pred:
                continue
            d = hamming(pts.desc[i], KF.desc[idx])
            if d < best:
                best, bidx = d, idx
        if bidx >= 0 and best <= 50:
            out[i] = bidx
            nf += 1
    return nf, np.array(out, np.int32)


def py_epipolar(kp1, kp2, F, sigma2):
    x1, y1, x2, y2 = F32(kp1["x"]), F32(kp1["y"]), F32(kp2["x"]), F32(kp2["y"])
    a = F32(fma32(x1, F[0], F32(y1 * F[3])) + F[6])
    b = F32(fma32(x1, F[1], F32(y1 * F[4])) + F[7])
    c = F32(fma32(y1, F[5], F32(x1 * F[2])) + F[8])
    num = F32(fma32(b, y2, F32(a * x2)) + c)
    den = fma32(a, a, F32(b * b))
    if den == 0:
        return False
    dsqr = F32(F32(num * num) / den)
    return F64(dsqr) < 3.84 * F64(sigma2[int(kp2["octave"])])


def py_triangulation(V1: View, h1, fv1, V2: View, h2, fv2, F12, check_ori):
    F = np.asarray(F12, F32).reshape(9)
    matched2 = [False] * V2.n
    m12 = [-1] * V1.n
    hist = [[] for _ in range(30)]
    nm = 0
    n2 = {int(n): k for k, n in enumerate(fv2.nodes)}
    for a, node in enumerate(fv1.nodes):
        b = n2.get(int(node))
        if b is None:
            continue
        for idx1 in fv1.features[fv1.offsets[a]:fv1.offsets[a + 1]]:
            if h1[idx1]:
                continue
            lst = []
            for idx2 in fv2.features[fv2.offsets[b]:fv2.offsets[b + 1]]:
                if matched2[idx2] or h2[idx2]:
                    continue
                d = hamming(V1.desc[idx1], V2.desc[idx2])
                if d > 50:
                    continue
                lst.append((d, int(idx2)))
            if not lst:
                continue
            lst.sort()
            th = 2 * lst[0][0]
            for d, idx2 in lst:
                if d > th:
                    break
                if py_epipolar(V1.kps[idx1], V2.kps[idx2], F, V2.mvLevelSigma2):
                    matched2[idx2] = True
                    m12[idx1] = idx2
                    nm += 1
                    if check_ori:
                        hist[rot_bin(V1.kps[idx1]["angle"], V2.kps[idx2]["angle"])].append(int(idx1))
                    break
    if check_ori:
        keep = three_maxima(hist)
        for i, h in enumerate(hist):
            if i in keep:
                continue
            for j in h:
                m12[j] = -1
                nm -= 1
    return nm, np.array(m12, np.int32)


@pytest.mark.parametrize("seed", range(4))
def test_window_search_vs_python(seed):
    rng = np.random.default_rng(seed)
    F2 = S.view(rng, 250, clusters=3, spread=15)
    idx = rng.integers(0, F2.n, 200)
    k1 = F2.kps[idx].copy()
    k1["x"] = np.clip(k1["x"] + rng.normal(0, 3, 200), 0, S.W - 1)
    k1["angle"] = (k1["angle"] + rng.choice([0, 0, 120], 200)) % 360
    F1 = View(k1, S.perturb(rng, F2.desc[idx], 80), (0, S.W, 0, S.H))
    u = (rng.random(200) < 0.9).astype(np.uint8)
    for args in ((60, 0, INT_MAX, 0.9, True), (100, 1, 4, 0.75, False)):
        ref = py_window_search(F1, u, F2, *args)
        n, m = OracleMatcher(args[3], args[4]).WindowSearch(F1, u, F2, *args[:3])
        assert n == ref[0] and n > 0
        np.testing.assert_array_equal(m, ref[1])


@pytest.mark.parametrize("seed", range(3))
def test_is_in_frustum_and_local_projection_vs_python(seed):
    rng = np.random.default_rng(10 + seed)
    F = S.view(rng, 250)
    mps, _ = S.map_points_on(rng, F, 300, bad_frac=0.3)
    o = OracleMatcher(0.8)
    iv, px, py, lv, vc = o.isInFrustum(F, mps, 0.5)
    ref = py_is_in_frustum(F, mps, 0.5)
    for i, r in enumerate(ref):
        assert iv[i] == r[0]
        if r[0]:
            assert (px[i], py[i], lv[i], vc[i]) == (r[1], r[2], r[3], r[4])
    taken = (rng.random(F.n) < 0.2).astype(np.uint8)
    for th in (1.0, 3.0):
        ref = py_sbp_local(F, taken, iv, px, py, lv, vc, mps.desc, th, 0.8)
        n, m = o.SearchByProjection_Local(F, taken, iv, px, py, lv, vc, mps.desc, th)
        assert n == ref[0] and n > 0
        np.testing.assert_array_equal(m, ref[1])


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("scw", [False, True])
def test_fuse_vs_python(seed, scw):
    rng = np.random.default_rng(20 + seed)
    KF = S.view(rng, 250)
    pts, _ = S.map_points_on(rng, KF, 300)
    u = (rng.random(pts.n) < 0.9).astype(np.uint8)
    ref = py_fuse(KF, pts, u, 3.0, scw)
    n, m = OracleMatcher().Fuse(KF, pts, u, 3.0, scw)
    assert n == ref[0] and n > 0
    np.testing.assert_array_equal(m, ref[1])


@pytest.mark.parametrize("seed", range(3))
def test_triangulation_vs_python(seed):
    rng = np.random.default_rng(30 + seed)
    V1, V2, P, i1, i2 = S.two_views_of_points(rng, 150, n_extra=80, kmax=45)
    ids = np.sort(rng.choice(10**5, 20, replace=False))
    a = rng.integers(0, 20, 150)
    a1 = rng.integers(0, 20, V1.n)
    a2 = rng.integers(0, 20, V2.n)
    a1[i1] = a
    a2[i2] = a
    fv1, _, _ = S.feature_vector(rng, V1.n, node_ids=ids, assign=a1)
    fv2, _, _ = S.feature_vector(rng, V2.n, node_ids=ids, assign=a2)
    F12 = S.fundamental12(V1, V2)
    h1 = (rng.random(V1.n) < 0.2).astype(np.uint8)
    h2 = (rng.random(V2.n) < 0.2).astype(np.uint8)
    for co in (True, False):
        ref = py_triangulation(V1, h1, fv1, V2, h2, fv2, F12, co)
        n, m = OracleMatcher(0.6, co).SearchForTriangulation(V1, h1, fv1, V2, h2, fv2, F12)
        assert n == ref[0] and n > 0
        np.testing.assert_array_equal(m, ref[1])


def test_keyframe_area_vs_python():
    rng = np.random.default_rng(5)
    V = S.view(rng, 400)
    P = PyView(V)
    o = OracleMatcher()
    for _ in range(200):
        x, y, r = rng.uniform(-30, 670), rng.uniform(-30, 510), rng.uniform(0, 80)
        assert list(o.GetFeaturesInArea(V, x, y, r, keyframe=True)) == P.kf_area(x, y, r)
        lo = int(rng.integers(-1, 8))
        hi = -1 if lo == -1 else int(min(7, lo + rng.integers(0, 3)))
        assert list(o.GetFeaturesInArea(V, x, y, r, lo, hi)) == P.area(x, y, r, lo, hi)
