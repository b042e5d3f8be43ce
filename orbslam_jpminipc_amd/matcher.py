"""ORBmatcher and Frame — host mirror of the reference classes over the HIP C ABI.

Reference: include/ORBmatcher.h:36-108, src/ORBmatcher.cc (SearchForInitialization
598-713, DescriptorDistance 1794-1810); include/Frame.h:43-138, src/Frame.cc (grid
bounds 73-86, 321-349).  Matching itself runs in the k_match_init HIP kernel.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import KEYPOINT_DTYPE, FrameBounds, check, hip_lib, ptr
from .views import FeatureVector, MapPointSet, View, flags


class Frame:
    """The matcher-facing part of ORB_SLAM::Frame: mvKeys, mvKeysUn, mDescriptors, image bounds.

    Without a camera, or with k1 == 0 (the configs' camera), mvKeysUn == mvKeys
    (Frame.cc:291-295) and the grid bounds are the image rectangle (Frame.cc:343-347).  With
    K and distCoef (k1, k2, p1, p2) and k1 != 0, mvKeysUn = UndistortKeyPoints (Frame.cc:297-318)
    and the bounds ComputeImageBounds (Frame.cc:323-340), both on the GPU (camera.py).
    """

    def __init__(self, keypoints: np.ndarray, descriptors, width: int, height: int, K=None, distCoef=None):
        self.mvKeys = np.asarray(keypoints, KEYPOINT_DTYPE)
        self.mvKeysUn = self.mvKeys
        self.N = len(self.mvKeys)
        self.mDescriptors = (np.zeros((0, 32), np.uint8) if descriptors is None
                             else np.ascontiguousarray(descriptors, np.uint8))
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = 0, int(width), 0, int(height)
        if (K is None) != (distCoef is None):
            raise ValueError("K and distCoef go together")
        if K is not None:
            from . import camera

            if self.N:
                self.mvKeysUn = camera.undistort_keypoints(self.mvKeys, K, distCoef)
            b = camera.image_bounds(width, height, K, distCoef)  # once per camera (Frame.cc:73-86)
            self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = b.min_x, b.max_x, b.min_y, b.max_y

    @classmethod
    def from_image(cls, image: np.ndarray, extractor, K=None, distCoef=None) -> "Frame":
        kps, desc = extractor(image)
        if kps is None:
            kps = np.zeros(0, KEYPOINT_DTYPE)
        return cls(kps, desc, image.shape[1], image.shape[0], K, distCoef)

    def bounds(self) -> FrameBounds:
        return FrameBounds(self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self._lib = hip_lib()
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return int(hip_lib().orb_descriptor_distance(ptr(a), ptr(b)))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray, vnMatches12: list,
                                windowSize: int = 10) -> int:
        """Returns nmatches; vnMatches12 is reassigned (N1 ints, -1 = none) and vbPrevMatched
        ((N1, 2) float32) updated in place, as in ORBmatcher.cc:598-713."""
        prev = vbPrevMatched
        if not (isinstance(prev, np.ndarray) and prev.dtype == np.float32 and prev.flags.c_contiguous
                and prev.shape == (F1.N, 2)):
            raise TypeError("vbPrevMatched must be a C-contiguous (N1, 2) float32 array")
        m12 = np.full(F1.N, -1, np.int32)
        n = ctypes.c_int()
        check(self._lib.orb_search_for_initialization(
            ptr(F1.mvKeysUn), ptr(F1.mDescriptors), F1.N, ptr(F2.mvKeysUn), ptr(F2.mDescriptors), F2.N,
            F1.bounds(), self.mfNNratio, int(self.mbCheckOrientation), int(windowSize), ptr(prev), ptr(m12),
            ctypes.byref(n)))
        vnMatches12[:] = m12.tolist()
        return n.value

    # ---- the rest of the family (csrc/orb_match.hip); views.View stands for Frame/KeyFrame ----
    # Map state the reference reads through MapPoint / KeyFrame methods arrives as flag
    # arrays (include/orb_abi.h names the condition of each); outputs are index arrays.
    # Every array handed to the C ABI is bound to a local first (ctypes keeps no reference).

    def SearchByBoW_KF_F(self, pKF: View, kf_usable, kf_fv: FeatureVector, F: View, f_fv: FeatureVector,
                         device: int = 0):
        """SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (ORBmatcher.cc:155-284).
        Returns (nmatches, f_match[N_F] = KF keypoint index or -1)."""
        out = np.full(F.n, -1, np.int32)
        u = flags(kf_usable, pKF.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_bow_kf_f(pKF.ref(), ptr(u), kf_fv.struct(), F.ref(), f_fv.struct(),
                                               self.mfNNratio, int(self.mbCheckOrientation), ptr(out),
                                               ctypes.byref(n), device))
        return n.value, out

    def SearchByBoW_KF_KF(self, pKF1: View, usable1, fv1: FeatureVector, pKF2: View, usable2, fv2: FeatureVector,
                          device: int = 0):
        """SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12) (ORBmatcher.cc:715-850).
        Returns (nmatches, match12[N1] = KF2 keypoint index or -1)."""
        out = np.full(pKF1.n, -1, np.int32)
        u1, u2 = flags(usable1, pKF1.n), flags(usable2, pKF2.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_bow_kf_kf(pKF1.ref(), ptr(u1), fv1.struct(), pKF2.ref(), ptr(u2),
                                                fv2.struct(), self.mfNNratio, int(self.mbCheckOrientation), ptr(out),
                                                ctypes.byref(n), device))
        return n.value, out

    def SearchForTriangulation(self, pKF1: View, has_mp1, fv1: FeatureVector, pKF2: View, has_mp2,
                               fv2: FeatureVector, F12, device: int = 0):
        """SearchForTriangulation(pKF1, pKF2, F12, ...) (ORBmatcher.cc:852-1014).
        Returns (nmatches, match12[N1]); vMatchedPairs = [(i, match12[i]) for match12[i] >= 0]."""
        out = np.full(pKF1.n, -1, np.int32)
        F = np.ascontiguousarray(np.asarray(F12, np.float32).reshape(9))
        h1 = np.zeros(pKF1.n, np.uint8) if has_mp1 is None else flags(has_mp1, pKF1.n)
        h2 = np.zeros(pKF2.n, np.uint8) if has_mp2 is None else flags(has_mp2, pKF2.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_for_triangulation(pKF1.ref(), ptr(h1), fv1.struct(), pKF2.ref(), ptr(h2),
                                                     fv2.struct(), ptr(F), self.mfNNratio,
                                                     int(self.mbCheckOrientation), ptr(out), ctypes.byref(n),
                                                     device))
        return n.value, out

    def WindowSearch(self, F1: View, usable1, F2: View, windowSize: int, minScaleLevel: int = 0,
                     maxScaleLevel: int = 2**31 - 1, device: int = 0):
        """WindowSearch (ORBmatcher.cc:409-516).  Returns (nmatches, match21[N2] = F1 index or -1)."""
        out = np.full(F2.n, -1, np.int32)
        u = flags(usable1, F1.n)
        n = ctypes.c_int()
        check(self._lib.orb_window_search(F1.ref(), ptr(u), F2.ref(), int(windowSize), int(minScaleLevel),
                                          int(maxScaleLevel), self.mfNNratio, int(self.mbCheckOrientation), ptr(out),
                                          ctypes.byref(n), device))
        return n.value, out

    def SearchByProjection_Local(self, F: View, f_taken, usable, proj_x, proj_y, level, view_cos, mp_desc,
                                 th: float = 1.0, device: int = 0):
        """SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:49-125) over
        isInFrustum output.  Returns (nmatches, f_match[N] = MapPoint row newly assigned or -1)."""
        m = len(proj_x)
        out = np.full(F.n, -1, np.int32)
        tk = np.zeros(F.n, np.uint8) if f_taken is None else flags(f_taken, F.n)
        u = flags(usable, m)
        a = [np.ascontiguousarray(np.asarray(x, t)) for x, t in
             ((proj_x, np.float32), (proj_y, np.float32), (level, np.int32), (view_cos, np.float32))]
        d = np.ascontiguousarray(np.asarray(mp_desc, np.uint8).reshape(-1, 32))
        n = ctypes.c_int()
        check(self._lib.orb_search_by_projection_local(F.ref(), ptr(tk), m, ptr(u), *map(ptr, a), ptr(d), float(th),
                                                       self.mfNNratio, ptr(out), ctypes.byref(n), device))
        return n.value, out

    def isInFrustum(self, F: View, mps: MapPointSet, viewingCosLimit: float = 0.5, device: int = 0):
        """Frame::isInFrustum (Frame.cc:137-198) for every MapPoint.
        Returns (in_view u8, proj_x, proj_y, level i32, view_cos)."""
        m = mps.n
        iv = np.zeros(m, np.uint8)
        px, py, vc = (np.zeros(m, np.float32) for _ in range(3))
        lv = np.zeros(m, np.int32)
        check(self._lib.orb_frame_is_in_frustum(F.ref(), mps.struct(), float(viewingCosLimit), ptr(iv), ptr(px),
                                                ptr(py), ptr(lv), ptr(vc), device))
        return iv, px, py, lv, vc

    def SearchByProjection_F2F(self, F1: View, mp1: MapPointSet, usable1, F2: View, f2_taken, windowSize: int,
                               device: int = 0):
        """SearchByProjection(Frame& F1, Frame& F2, windowSize, ...) (ORBmatcher.cc:519-594).
        Returns (nmatches, match2[N2] = F1 index newly assigned or -1)."""
        out = np.full(F2.n, -1, np.int32)
        u = flags(usable1, F1.n)
        tk = np.zeros(F2.n, np.uint8) if f2_taken is None else flags(f2_taken, F2.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_projection_f2f(F1.ref(), mp1.struct(), ptr(u), F2.ref(), ptr(tk),
                                                     int(windowSize), self.mfNNratio, ptr(out), ctypes.byref(n),
                                                     device))
        return n.value, out

    def SearchByProjection_Motion(self, Cur: View, cur_taken, Last: View, mp: MapPointSet, usable, th: float,
                                  device: int = 0):
        """SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th) (1507-1620).
        Returns (nmatches, cur_match[N] = LastFrame index newly assigned or -1)."""
        out = np.full(Cur.n, -1, np.int32)
        tk = np.zeros(Cur.n, np.uint8) if cur_taken is None else flags(cur_taken, Cur.n)
        u = flags(usable, Last.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_projection_motion(Cur.ref(), ptr(tk), Last.ref(), mp.struct(), ptr(u),
                                                        float(th), int(self.mbCheckOrientation), ptr(out),
                                                        ctypes.byref(n), device))
        return n.value, out

    def SearchByProjection_Reloc(self, Cur: View, cur_taken, pKF: View, mp: MapPointSet, usable, th: float,
                                 ORBdist: int, device: int = 0):
        """SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (1622-1746)."""
        out = np.full(Cur.n, -1, np.int32)
        tk = np.zeros(Cur.n, np.uint8) if cur_taken is None else flags(cur_taken, Cur.n)
        u = flags(usable, pKF.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_projection_reloc(Cur.ref(), ptr(tk), pKF.ref(), mp.struct(), ptr(u),
                                                       float(th), int(ORBdist), int(self.mbCheckOrientation),
                                                       ptr(out), ctypes.byref(n), device))
        return n.value, out

    def SearchByProjection_Sim3(self, pKF: View, kf_taken, pts: MapPointSet, usable, th: int, device: int = 0):
        """SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:286-407);
        pKF carries the Scw decomposition as its pose.  Returns (nmatches, kf_match[N])."""
        out = np.full(pKF.n, -1, np.int32)
        tk = np.zeros(pKF.n, np.uint8) if kf_taken is None else flags(kf_taken, pKF.n)
        u = flags(usable, pts.n)
        n = ctypes.c_int()
        check(self._lib.orb_search_by_projection_sim3(pKF.ref(), ptr(tk), pts.struct(), ptr(u), int(th), ptr(out),
                                                      ctypes.byref(n), device))
        return n.value, out

    def SearchBySim3(self, pKF1: View, mp1: MapPointSet, usable1, pKF2: View, mp2: MapPointSet, usable2, sR12,
                     t12, sR21, t21, th: float, device: int = 0):
        """SearchBySim3 (ORBmatcher.cc:1267-1505).  Returns (nFound, match12[N1])."""
        out = np.full(pKF1.n, -1, np.int32)
        u1, u2 = flags(usable1, pKF1.n), flags(usable2, pKF2.n)
        a = [np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1)) for x in (sR12, t12, sR21, t21)]
        n = ctypes.c_int()
        check(self._lib.orb_search_by_sim3(pKF1.ref(), mp1.struct(), ptr(u1), pKF2.ref(), mp2.struct(), ptr(u2),
                                           *map(ptr, a), float(th), ptr(out), ctypes.byref(n), device))
        return n.value, out

    def Fuse(self, pKF: View, pts: MapPointSet, usable, th: float = 2.5, scw: bool = False, device: int = 0):
        """Fuse(KeyFrame*, vector<MapPoint*>, th) (1016-1134) / Fuse(KeyFrame*, Scw, ...)
        (1136-1265).  Returns (nFused, best_idx[n_points])."""
        out = np.full(pts.n, -1, np.int32)
        u = flags(usable, pts.n)
        n = ctypes.c_int()
        check(self._lib.orb_fuse(pKF.ref(), pts.struct(), ptr(u), float(th), int(bool(scw)), ptr(out),
                                 ctypes.byref(n), device))
        return n.value, out

    @staticmethod
    def GetFeaturesInArea(view: View, x, y, r, min_level=None, max_level=None, keyframe: bool = False,
                          capacity: int = 1 << 20, device: int = 0):
        """Frame::GetFeaturesInArea (Frame.cc:200-265) / KeyFrame::GetFeaturesInArea
        (KeyFrame.cc:612-652) for a batch of windows; returns a list of index arrays."""
        x = np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1))
        q = len(x)
        y = np.ascontiguousarray(np.asarray(y, np.float32).reshape(-1))
        r = np.ascontiguousarray(np.broadcast_to(np.asarray(r, np.float32), (q,)))
        lo = hi = None
        if min_level is not None:
            lo = np.ascontiguousarray(np.broadcast_to(np.asarray(min_level, np.int32), (q,)))
            hi = np.ascontiguousarray(np.broadcast_to(np.asarray(max_level, np.int32), (q,)))
        off = np.zeros(q + 1, np.int32)
        out = np.zeros(max(capacity, 1), np.int32)
        check(hip_lib().orb_features_in_area(view.ref(), int(keyframe), q, ptr(x), ptr(y), ptr(r), ptr(lo), ptr(hi),
                                             ptr(off), ptr(out), capacity, device))
        return [out[off[i]:off[i + 1]].copy() for i in range(q)]

    def search_for_initialization_batch_device(self, d_kps, d_desc, d_counts, pair_f1, pair_f2, width: int,
                                               height: int, windowSize: int = 100, d_prev_xy=None, stream=None,
                                               bounds=None):
        """Batched SearchForInitialization over device extractor output (one wave per pair).

        d_kps (B, cap, 28) / d_desc (B, cap, 32) / d_counts (B,) as returned by
        ORBextractor.extract_batch_device (or mvKeysUn from camera.undistort_keypoints_batch_device,
        with `bounds` = camera.compute_image_bounds; default: the image rectangle);
        pair_f1 / pair_f2 int32 device tensors (P,).
        Returns (d_matches12 (P, cap) int32, d_nmatches (P,) int32).
        """
        import torch

        P = int(pair_f1.shape[0])
        cap = int(d_kps.shape[1])
        dev = d_kps.device
        m12 = torch.empty((P, cap), dtype=torch.int32, device=dev)
        nm = torch.empty((P,), dtype=torch.int32, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.orb_search_for_initialization_batch_device(
            ptr(d_kps), ptr(d_desc), ptr(d_counts), cap, P, ptr(pair_f1), ptr(pair_f2),
            bounds if bounds is not None else FrameBounds(0, width, 0, height), self.mfNNratio, int(self.mbCheckOrientation), int(windowSize),
            ptr(d_prev_xy), ptr(m12), ptr(nm), ctypes.c_void_p(s.cuda_stream)))
        return m12, nm

    def search_by_bow_batch_device(self, kf_kf: bool, d_kps, d_desc, d_counts, fv: dict, pair_a, pair_b,
                                   d_usable=None, stream=None):
        """SearchByBoW over many pairs in one launch (orb_search_by_bow_batch_device).

        d_kps (B, cap, 28) / d_desc (B, cap, 32) / d_counts (B,) as ORBextractor.extract_batch_device
        returns them; `fv` = ORBVocabulary.transform_batch_device's dict for the same frames;
        pair_a / pair_b int32 device tensors (P,): the KeyFrame (KF1) and the Frame (KF2) of each
        pair.  kf_kf False: SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:155-284), row p of the
        result = vpMapPointMatches over frame b's keypoints (frame-a keypoint index or -1); True:
        SearchByBoW(KeyFrame*, KeyFrame*) (715-850), row p = vpMatches12 over frame a's keypoints.
        d_usable (B, cap) uint8 or None (every keypoint has a usable MapPoint).
        Returns (d_match (P, cap) int32, d_nmatches (P,) int32).
        """
        import torch

        P = int(pair_a.shape[0])
        cap = int(d_kps.shape[1])
        dev = d_kps.device
        m = torch.empty((P, cap), dtype=torch.int32, device=dev)
        n = torch.empty((P,), dtype=torch.int32, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.orb_search_by_bow_batch_device(
            int(bool(kf_kf)), ptr(d_kps), ptr(d_desc), ptr(d_counts), cap, ptr(fv["fv_nodes"]), ptr(fv["fv_offsets"]),
            ptr(fv["fv_features"]), ptr(fv["fv_n"]), P, ptr(pair_a), ptr(pair_b), ptr(d_usable), self.mfNNratio,
            int(self.mbCheckOrientation), ptr(m), ptr(n), ctypes.c_void_p(s.cuda_stream)))
        return m, n
