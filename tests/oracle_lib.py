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


def search_for_initialization(k1, d1, k2, d2, width, height, prev, nnratio=0.9, checkOri=True, window=100):
    """Oracle SearchForInitialization (ORBmatcher.cc:598-713); prev updated in place."""
    L = lib()
    k1 = np.ascontiguousarray(k1, KEYPOINT_DTYPE)
    k2 = np.ascontiguousarray(k2, KEYPOINT_DTYPE)
    d1 = np.ascontiguousarray(d1, np.uint8)
    d2 = np.ascontiguousarray(d2, np.uint8)
    m12 = np.full(len(k1), -1, np.int32)
    n = ctypes.c_int()
    st = L.oracle_search_for_initialization(_p(k1), _p(d1), len(k1), _p(k2), _p(d2), len(k2),
                                            _Bounds(0, width, 0, height), nnratio, int(checkOri), window, _p(prev),
                                            _p(m12), ctypes.byref(n))
    assert st == 0
    return n.value, m12
