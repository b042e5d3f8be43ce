"""POD views the matcher family reads: Frame / KeyFrame, MapPoint arrays, FeatureVectors.

Host mirror of the C ABI structs of include/orb_abi.h (orb_frame_view_t, orb_map_points_t,
orb_feature_vector_t).  Each view keeps the numpy arrays its struct points at alive.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import KEYPOINT_DTYPE, MAX_VIEW_LEVELS, FeatureVectorCSR, FrameBounds, FrameView, MapPoints, ptr


def frame_scale_tables(nlevels: int, scale_factor: float):
    """mvScaleFactors / mvLevelSigma2 exactly as Frame::Frame builds them (Frame.cc:95-103):
    a float recurrence on mfScaleFactor = (float) ORBextractor::GetScaleFactor()."""
    f = np.float32(scale_factor)
    sf = np.zeros(MAX_VIEW_LEVELS, np.float32)
    s2 = np.zeros(MAX_VIEW_LEVELS, np.float32)
    sf[0] = np.float32(1.0)
    s2[0] = np.float32(1.0)
    for i in range(1, nlevels):
        sf[i] = np.float32(sf[i - 1] * f)
        s2[i] = np.float32(sf[i] * sf[i])
    return sf, s2


def camera_center(Rcw, tcw) -> np.ndarray:
    """Ow = -Rcw^T tcw (Frame::UpdatePoseMatrices, Frame.cc:130-135), accumulated in double as
    OpenCV's generic gemm does for CV_32F, rounded to float."""
    R = np.asarray(Rcw, np.float64).reshape(3, 3)
    t = np.asarray(tcw, np.float64).reshape(3)
    return (-(R.T @ t)).astype(np.float32)


class View:
    """A Frame or KeyFrame for the matchers (orb_frame_view_t)."""

    def __init__(self, keypoints, descriptors, bounds=(0, 640, 0, 480), nlevels: int = 8,
                 scale_factor: float = 1.2, calib=(500.0, 500.0, 320.0, 240.0), Rcw=None, tcw=None, Ow=None,
                 scale_factors=None, level_sigma2=None):
        self.kps = np.ascontiguousarray(np.asarray(keypoints, KEYPOINT_DTYPE))
        self.desc = np.ascontiguousarray(np.asarray(descriptors, np.uint8).reshape(-1, 32))
        if len(self.kps) != len(self.desc):
            raise ValueError("keypoints and descriptors differ in length")
        self.n = len(self.kps)
        self.nlevels = int(nlevels)
        if scale_factors is None:
            sf, s2 = frame_scale_tables(nlevels, scale_factor)
        else:
            sf = np.zeros(MAX_VIEW_LEVELS, np.float32)
            s2 = np.zeros(MAX_VIEW_LEVELS, np.float32)
            sf[:nlevels] = scale_factors
            s2[:nlevels] = level_sigma2
        self.mvScaleFactors = sf
        self.mvLevelSigma2 = s2
        self.bounds = tuple(int(b) for b in bounds)
        self.fx, self.fy, self.cx, self.cy = (np.float32(c) for c in calib)
        self.Rcw = np.eye(3, dtype=np.float32) if Rcw is None else np.asarray(Rcw, np.float32).reshape(3, 3)
        self.tcw = np.zeros(3, np.float32) if tcw is None else np.asarray(tcw, np.float32).reshape(3)
        self.Ow = camera_center(self.Rcw, self.tcw) if Ow is None else np.asarray(Ow, np.float32).reshape(3)

    def struct(self) -> FrameView:
        v = FrameView()
        v.kps = ptr(self.kps).value
        v.desc = ptr(self.desc).value
        v.n = self.n
        v.nlevels = self.nlevels
        v.bounds = FrameBounds(*[self.bounds[i] for i in (0, 1, 2, 3)])
        v.scale_factors[:] = [float(x) for x in self.mvScaleFactors]
        v.level_sigma2[:] = [float(x) for x in self.mvLevelSigma2]
        v.fx, v.fy, v.cx, v.cy = float(self.fx), float(self.fy), float(self.cx), float(self.cy)
        v.Rcw[:] = [float(x) for x in self.Rcw.reshape(9)]
        v.tcw[:] = [float(x) for x in self.tcw]
        v.Ow[:] = [float(x) for x in self.Ow]
        return v

    def ref(self):
        self._s = self.struct()
        return ctypes.byref(self._s)


class MapPointSet:
    """MapPoint attributes by row (orb_map_points_t); absent fields stay NULL."""

    def __init__(self, pos, normal=None, dmin=None, dmax=None, desc=None):
        self.pos = np.ascontiguousarray(np.asarray(pos, np.float32).reshape(-1, 3))
        self.n = len(self.pos)
        self.normal = None if normal is None else np.ascontiguousarray(np.asarray(normal, np.float32).reshape(-1, 3))
        self.dmin = None if dmin is None else np.ascontiguousarray(np.asarray(dmin, np.float32).reshape(-1))
        self.dmax = None if dmax is None else np.ascontiguousarray(np.asarray(dmax, np.float32).reshape(-1))
        self.desc = None if desc is None else np.ascontiguousarray(np.asarray(desc, np.uint8).reshape(-1, 32))

    def struct(self) -> MapPoints:
        return MapPoints(ptr(self.pos).value, ptr(self.normal).value, ptr(self.dmin).value, ptr(self.dmax).value,
                         ptr(self.desc).value, self.n)


class FeatureVector:
    """DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR."""

    def __init__(self, nodes, offsets, features):
        self.nodes = np.ascontiguousarray(np.asarray(nodes, np.uint32))
        self.offsets = np.ascontiguousarray(np.asarray(offsets, np.int32))
        self.features = np.ascontiguousarray(np.asarray(features, np.int32))
        if len(self.offsets) != len(self.nodes) + 1:
            raise ValueError("offsets must have n_nodes + 1 entries")

    @classmethod
    def from_dict(cls, d: dict) -> "FeatureVector":
        nodes = sorted(d)
        off = [0]
        feat = []
        for k in nodes:
            feat.extend(d[k])
            off.append(len(feat))
        return cls(nodes, off, feat)

    def struct(self) -> FeatureVectorCSR:
        return FeatureVectorCSR(ptr(self.nodes).value, ptr(self.offsets).value, ptr(self.features).value,
                                len(self.nodes))


def flags(a, n: int) -> np.ndarray:
    """Per-element uint8 flag array (None -> all set)."""
    if a is None:
        return np.ones(n, np.uint8)
    a = np.ascontiguousarray(np.asarray(a, np.uint8).reshape(-1))
    if len(a) != n:
        raise ValueError(f"flag array has {len(a)} entries, expected {n}")
    return a
