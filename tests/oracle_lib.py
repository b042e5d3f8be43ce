"""TEST INFRASTRUCTURE: ctypes wrapper of oracle/liborb_oracle.so (the CPU parity checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
ORACLE_PATH = ROOT / "oracle" / "liborb_oracle.so"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                           ("octave", "<i4"), ("class_id", "<i4")])


class _Bounds(ctypes.Structure):
    _fields_ = [("min_x", ctypes.c_int), ("max_x", ctypes.c_int), ("min_y", ctypes.c_int), ("max_y", ctypes.c_int)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(ORACLE_PATH))
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.oracle_extractor_create.restype = vp
        L.oracle_extractor_create.argtypes = [i, f, i, i, i]
        L.oracle_extractor_destroy.argtypes = [vp]
        L.oracle_get_level_info.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_extract.argtypes = [vp, vp, i, i, i, vp, i, vp, ctypes.POINTER(i)]
        L.oracle_level_image.argtypes = [vp, i, vp, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.oracle_level_blurred.argtypes = [vp, i, vp]
        L.oracle_cell_counts.argtypes = [vp, i, ctypes.POINTER(i), ctypes.POINTER(i), vp, i]
        L.oracle_fast_atan2.restype = f
        L.oracle_fast_atan2.argtypes = [f, f]
        L.oracle_sinf.restype = f
        L.oracle_sinf.argtypes = [f]
        L.oracle_cosf.restype = f
        L.oracle_cosf.argtypes = [f]
        L.oracle_descriptor_distance.argtypes = [vp, vp]
        L.oracle_nth_element_greater.argtypes = [vp, vp, i, i]
        L.oracle_gaussian_taps.argtypes = [vp]
        L.oracle_search_for_initialization.argtypes = [vp, vp, i, vp, vp, i, _Bounds, f, i, i, vp, vp,
                                                       ctypes.POINTER(i)]
        L.oracle_features_in_area.argtypes = [vp, i, _Bounds, f, f, f, i, i, vp, i]
        L.oracle_search_by_bow_kf_f.argtypes = [vp, vp, i, vp, vp, vp, vp, i, vp, vp, i, vp, vp, vp, i, f, i, vp,
                                                ctypes.POINTER(i)]
        L.oracle_search_by_bow_kf_kf.argtypes = [vp, vp, i, vp, vp, vp, vp, i, vp, vp, i, vp, vp, vp, vp, i, f, i,
                                                 vp, ctypes.POINTER(i)]
        L.oracle_rot_bin.argtypes = [f, f]
        L.oracle_resize.argtypes = [vp, i, i, i, vp, i, i, i]
        L.oracle_blur_padded.argtypes = [vp, i, i, vp]
        L.oracle_fast.argtypes = [vp, i, i, i, i, vp, i]
        L.oracle_undistort_points.argtypes = [vp, vp, vp, i, vp]
        L.oracle_undistort_keypoints.argtypes = [vp, i, vp, vp, vp]
        L.oracle_compute_image_bounds.argtypes = [i, i, vp, vp, ctypes.POINTER(_Bounds)]
        L.oracle_bench.restype = ctypes.c_double
        L.oracle_bench.argtypes = [i, f, i, i, vp, i, i, i, i, ctypes.c_int64, i, i, ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(ctypes.c_int64)]
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


class Oracle:
    """CPU restatement of ORB_SLAM::ORBextractor + the matcher core (oracle/orb_oracle.cpp)."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, scoreType=1, fastTh=20):
        self.L = lib()
        self.h = self.L.oracle_extractor_create(nfeatures, scaleFactor, nlevels, scoreType, fastTh)
        assert self.h, "oracle_extractor_create failed"
        self.nlevels = nlevels
        fpl = np.zeros(nlevels, np.int32)
        self.L.oracle_get_level_info(self.h, _p(fpl), None, None, None)
        self.cap = int(fpl.sum()) + 16

    def __del__(self):
        try:
            self.L.oracle_extractor_destroy(self.h)
        except Exception:
            pass

    def level_info(self):
        fpl = np.zeros(self.nlevels, np.int32)
        sf = np.zeros(self.nlevels, np.float32)
        isf = np.zeros(self.nlevels, np.float32)
        um = np.zeros(16, np.int32)
        self.L.oracle_get_level_info(self.h, _p(fpl), _p(sf), _p(isf), _p(um))
        return fpl, sf, isf, um

    def extract(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        kps = np.empty(self.cap, KEYPOINT_DTYPE)
        desc = np.empty((self.cap, 32), np.uint8)
        n = ctypes.c_int()
        st = self.L.oracle_extract(self.h, _p(img), w, h, w, _p(kps), self.cap, _p(desc), ctypes.byref(n))
        if st != 0:
            raise RuntimeError(f"oracle_extract status {st}")
        n = n.value
        return kps[:n].copy(), desc[:n].copy()

    def level_image(self, l: int):
        w, h = ctypes.c_int(), ctypes.c_int()
        self.L.oracle_level_image(self.h, l, None, ctypes.byref(w), ctypes.byref(h))
        out = np.empty((h.value + 32, w.value + 32), np.uint8)
        self.L.oracle_level_image(self.h, l, _p(out), ctypes.byref(w), ctypes.byref(h))
        return out

    def cell_counts(self, l: int):
        rows, cols = ctypes.c_int(), ctypes.c_int()
        out = np.zeros(4096, np.int32)
        n = self.L.oracle_cell_counts(self.h, l, ctypes.byref(rows), ctypes.byref(cols), _p(out), 4096)
        return out[:n].reshape(rows.value, cols.value)

    @staticmethod
    def search_for_initialization(k1, d1, k2, d2, width, height, prev, nnratio=0.9, checkOri=True, window=100):
        return search_for_initialization(k1, d1, k2, d2, width, height, prev, nnratio, checkOri, window)


def search_for_initialization(k1, d1, k2, d2, width, height, prev, nnratio=0.9, checkOri=True, window=100,
                              bounds=None):
    """Oracle SearchForInitialization (ORBmatcher.cc:598-713); prev updated in place.  `bounds`
    = (min_x, max_x, min_y, max_y) of the frame grid (default: the image rectangle)."""
    L = lib()
    k1 = np.ascontiguousarray(k1, KEYPOINT_DTYPE)
    k2 = np.ascontiguousarray(k2, KEYPOINT_DTYPE)
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    m12 = np.full(len(k1), -1, np.int32)
    n = ctypes.c_int()
    st = L.oracle_search_for_initialization(_p(k1), _p(d1), len(k1), _p(k2), _p(d2), len(k2),
                                            _Bounds(*(bounds or (0, width, 0, height))), nnratio, int(checkOri), window, _p(prev),
                                            _p(m12), ctypes.byref(n))
    assert st == 0
    return n.value, m12


# ---- Frame::UndistortKeyPoints / ComputeImageBounds (oracle/orb_oracle_frame.cpp) ----------
def undistort_points(xy, K4, dist4):
    xy = np.ascontiguousarray(np.asarray(xy, np.float32).reshape(-1, 2))
    out = np.empty_like(xy)
    k, d = np.ascontiguousarray(K4, np.float32), np.ascontiguousarray(dist4, np.float32)
    assert lib().oracle_undistort_points(_p(k), _p(d), _p(xy), len(xy), _p(out)) == 0
    return out


def undistort_keypoints(kps, K4, dist4):
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.empty_like(kps)
    k, d = np.ascontiguousarray(K4, np.float32), np.ascontiguousarray(dist4, np.float32)
    assert lib().oracle_undistort_keypoints(_p(kps), len(kps), _p(k), _p(d), _p(out)) == 0
    return out


def compute_image_bounds(cols, rows, K4, dist4):
    b = _Bounds()
    k, d = np.ascontiguousarray(K4, np.float32), np.ascontiguousarray(dist4, np.float32)
    assert lib().oracle_compute_image_bounds(cols, rows, _p(k), _p(d), ctypes.byref(b)) == 0
    return (b.min_x, b.max_x, b.min_y, b.max_y)


# ---- the rest of the ORBmatcher family (oracle/orb_oracle_match.cpp) -----------------------
def _bind_family(L):
    from orbslam_jpminipc_amd._native import FeatureVectorCSR, FrameView, MapPoints

    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    pv, pi = ctypes.POINTER(FrameView), ctypes.POINTER(ctypes.c_int)
    sig = {
        "oracle_features_in_area_view": [pv, i, f, f, f, i, i, vp, i],
        "oracle_frame_is_in_frustum": [pv, MapPoints, f, vp, vp, vp, vp, vp],
        "oracle_search_by_projection_local": [pv, vp, i, vp, vp, vp, vp, vp, vp, f, f, vp, pi],
        "oracle_window_search": [pv, vp, pv, i, i, i, f, i, vp, pi],
        "oracle_search_by_projection_f2f": [pv, MapPoints, vp, pv, vp, i, f, vp, pi],
        "oracle_search_by_projection_motion": [pv, vp, pv, MapPoints, vp, f, i, vp, pi],
        "oracle_search_by_projection_reloc": [pv, vp, pv, MapPoints, vp, f, i, i, vp, pi],
        "oracle_search_by_projection_sim3": [pv, vp, MapPoints, vp, i, vp, pi],
        "oracle_fuse": [pv, MapPoints, vp, f, i, vp, pi],
        "oracle_search_by_sim3": [pv, MapPoints, vp, pv, MapPoints, vp, vp, vp, vp, vp, f, vp, pi],
        "oracle_search_for_triangulation": [pv, vp, FeatureVectorCSR, pv, vp, FeatureVectorCSR, vp, f, i, vp, pi],
    }
    for k, a in sig.items():
        getattr(L, k).argtypes = a
        getattr(L, k).restype = i


class OracleMatcher:
    """CPU restatement with the same method surface as orbslam_jpminipc_amd.ORBmatcher's
    family methods (views.View / MapPointSet / FeatureVector in, (n, index array) out)."""

    def __init__(self, nnratio=0.6, checkOri=True):
        self.L = lib()
        if not getattr(self.L, "_family_bound", False):
            _bind_family(self.L)
            self.L._family_bound = True
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def _u8(a, n, default=1):
        if a is None:
            return np.full(n, default, np.uint8)
        return np.ascontiguousarray(np.asarray(a, np.uint8).reshape(-1))

    def SearchByBoW_KF_F(self, KF, kf_usable, kf_fv, F, f_fv):
        out = np.full(F.n, -1, np.int32)
        n = ctypes.c_int()
        u = self._u8(kf_usable, KF.n)
        st = self.L.oracle_search_by_bow_kf_f(_p(KF.kps), _p(KF.desc), KF.n, _p(u), _p(kf_fv.nodes),
                                              _p(kf_fv.offsets), _p(kf_fv.features), len(kf_fv.nodes), _p(F.kps),
                                              _p(F.desc), F.n, _p(f_fv.nodes), _p(f_fv.offsets), _p(f_fv.features),
                                              len(f_fv.nodes), self.mfNNratio, int(self.mbCheckOrientation),
                                              _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchByBoW_KF_KF(self, KF1, usable1, fv1, KF2, usable2, fv2):
        out = np.full(KF1.n, -1, np.int32)
        n = ctypes.c_int()
        u1, u2 = self._u8(usable1, KF1.n), self._u8(usable2, KF2.n)
        st = self.L.oracle_search_by_bow_kf_kf(_p(KF1.kps), _p(KF1.desc), KF1.n, _p(u1), _p(fv1.nodes),
                                               _p(fv1.offsets), _p(fv1.features), len(fv1.nodes), _p(KF2.kps),
                                               _p(KF2.desc), KF2.n, _p(u2), _p(fv2.nodes), _p(fv2.offsets),
                                               _p(fv2.features), len(fv2.nodes), self.mfNNratio,
                                               int(self.mbCheckOrientation), _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchForTriangulation(self, KF1, has_mp1, fv1, KF2, has_mp2, fv2, F12):
        out = np.full(KF1.n, -1, np.int32)
        n = ctypes.c_int()
        h1, h2 = self._u8(has_mp1, KF1.n, 0), self._u8(has_mp2, KF2.n, 0)
        F = np.ascontiguousarray(np.asarray(F12, np.float32).reshape(9))
        st = self.L.oracle_search_for_triangulation(KF1.ref(), _p(h1), fv1.struct(), KF2.ref(), _p(h2),
                                                    fv2.struct(), _p(F), self.mfNNratio,
                                                    int(self.mbCheckOrientation), _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def WindowSearch(self, F1, usable1, F2, windowSize, minScaleLevel=0, maxScaleLevel=2**31 - 1):
        out = np.full(F2.n, -1, np.int32)
        n = ctypes.c_int()
        u = self._u8(usable1, F1.n)
        st = self.L.oracle_window_search(F1.ref(), _p(u), F2.ref(), int(windowSize), int(minScaleLevel),
                                         int(maxScaleLevel), self.mfNNratio, int(self.mbCheckOrientation), _p(out),
                                         ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchByProjection_Local(self, F, f_taken, usable, proj_x, proj_y, level, view_cos, mp_desc, th=1.0):
        m = len(proj_x)
        out = np.full(F.n, -1, np.int32)
        n = ctypes.c_int()
        tk, u = self._u8(f_taken, F.n, 0), self._u8(usable, m)
        a = [np.ascontiguousarray(np.asarray(x, t)) for x, t in
             ((proj_x, np.float32), (proj_y, np.float32), (level, np.int32), (view_cos, np.float32))]
        d = np.ascontiguousarray(np.asarray(mp_desc, np.uint8).reshape(-1, 32))
        st = self.L.oracle_search_by_projection_local(F.ref(), _p(tk), m, _p(u), *map(_p, a), _p(d), float(th),
                                                      self.mfNNratio, _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def isInFrustum(self, F, mps, viewingCosLimit=0.5):
        m = mps.n
        iv = np.zeros(m, np.uint8)
        px, py, vc = (np.zeros(m, np.float32) for _ in range(3))
        lv = np.zeros(m, np.int32)
        st = self.L.oracle_frame_is_in_frustum(F.ref(), mps.struct(), float(viewingCosLimit), _p(iv), _p(px), _p(py),
                                               _p(lv), _p(vc))
        assert st == 0
        return iv, px, py, lv, vc

    def SearchByProjection_F2F(self, F1, mp1, usable1, F2, f2_taken, windowSize):
        out = np.full(F2.n, -1, np.int32)
        n = ctypes.c_int()
        u, tk = self._u8(usable1, F1.n), self._u8(f2_taken, F2.n, 0)
        st = self.L.oracle_search_by_projection_f2f(F1.ref(), mp1.struct(), _p(u), F2.ref(), _p(tk),
                                                    int(windowSize), self.mfNNratio, _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchByProjection_Motion(self, Cur, cur_taken, Last, mp, usable, th):
        out = np.full(Cur.n, -1, np.int32)
        n = ctypes.c_int()
        tk, u = self._u8(cur_taken, Cur.n, 0), self._u8(usable, Last.n)
        st = self.L.oracle_search_by_projection_motion(Cur.ref(), _p(tk), Last.ref(), mp.struct(), _p(u), float(th),
                                                       int(self.mbCheckOrientation), _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchByProjection_Reloc(self, Cur, cur_taken, KF, mp, usable, th, ORBdist):
        out = np.full(Cur.n, -1, np.int32)
        n = ctypes.c_int()
        tk, u = self._u8(cur_taken, Cur.n, 0), self._u8(usable, KF.n)
        st = self.L.oracle_search_by_projection_reloc(Cur.ref(), _p(tk), KF.ref(), mp.struct(), _p(u), float(th),
                                                      int(ORBdist), int(self.mbCheckOrientation), _p(out),
                                                      ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchByProjection_Sim3(self, KF, kf_taken, pts, usable, th):
        out = np.full(KF.n, -1, np.int32)
        n = ctypes.c_int()
        tk, u = self._u8(kf_taken, KF.n, 0), self._u8(usable, pts.n)
        st = self.L.oracle_search_by_projection_sim3(KF.ref(), _p(tk), pts.struct(), _p(u), int(th), _p(out),
                                                     ctypes.byref(n))
        assert st == 0
        return n.value, out

    def SearchBySim3(self, KF1, mp1, usable1, KF2, mp2, usable2, sR12, t12, sR21, t21, th):
        out = np.full(KF1.n, -1, np.int32)
        n = ctypes.c_int()
        u1, u2 = self._u8(usable1, KF1.n), self._u8(usable2, KF2.n)
        a = [np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1)) for x in (sR12, t12, sR21, t21)]
        st = self.L.oracle_search_by_sim3(KF1.ref(), mp1.struct(), _p(u1), KF2.ref(), mp2.struct(), _p(u2),
                                          *map(_p, a), float(th), _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def Fuse(self, KF, pts, usable, th=2.5, scw=False):
        out = np.full(pts.n, -1, np.int32)
        n = ctypes.c_int()
        u = self._u8(usable, pts.n)
        st = self.L.oracle_fuse(KF.ref(), pts.struct(), _p(u), float(th), int(bool(scw)), _p(out), ctypes.byref(n))
        assert st == 0
        return n.value, out

    def GetFeaturesInArea(self, view, x, y, r, min_level=-1, max_level=-1, keyframe=False):
        out = np.zeros(max(view.n, 1), np.int32)
        k = self.L.oracle_features_in_area_view(view.ref(), int(keyframe), float(x), float(y), float(r),
                                                int(min_level), int(max_level), _p(out), len(out))
        assert k >= 0
        return out[:k].copy()
