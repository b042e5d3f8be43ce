"""ORBmatcher and Frame — host mirror of the reference classes over the HIP C ABI.

Reference: include/ORBmatcher.h:36-108, src/ORBmatcher.cc (SearchForInitialization
598-713, DescriptorDistance 1794-1810); include/Frame.h:43-138, src/Frame.cc (grid
bounds 73-86, 321-349).  Matching itself runs in the k_match_init HIP kernel.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import KEYPOINT_DTYPE, FrameBounds, check, hip_lib, ptr


class Frame:
    """The matcher-facing part of ORB_SLAM::Frame: mvKeysUn, mDescriptors, image bounds.

    With zero distortion (k1 == 0, the configs' camera) mvKeysUn == mvKeys (Frame.cc:291-295)
    and the grid bounds are the image rectangle (Frame.cc:343-347).
    """

    def __init__(self, keypoints: np.ndarray, descriptors, width: int, height: int):
        self.mvKeys = np.asarray(keypoints, KEYPOINT_DTYPE)
        self.mvKeysUn = self.mvKeys
        self.N = len(self.mvKeys)
        self.mDescriptors = (np.zeros((0, 32), np.uint8) if descriptors is None
                             else np.ascontiguousarray(descriptors, np.uint8))
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = 0, int(width), 0, int(height)

    @classmethod
    def from_image(cls, image: np.ndarray, extractor) -> "Frame":
        kps, desc = extractor(image)
        if kps is None:
            kps = np.zeros(0, KEYPOINT_DTYPE)
        return cls(kps, desc, image.shape[1], image.shape[0])

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

    def search_for_initialization_batch_device(self, d_kps, d_desc, d_counts, pair_f1, pair_f2, width: int,
                                               height: int, windowSize: int = 100, d_prev_xy=None, stream=None):
        """Batched SearchForInitialization over device extractor output (one wave per pair).

        d_kps (B, cap, 28) / d_desc (B, cap, 32) / d_counts (B,) as returned by
        ORBextractor.extract_batch_device; pair_f1 / pair_f2 int32 device tensors (P,).
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
            FrameBounds(0, width, 0, height), self.mfNNratio, int(self.mbCheckOrientation), int(windowSize),
            ptr(d_prev_xy), ptr(m12), ptr(nm), ctypes.c_void_p(s.cuda_stream)))
        return m12, nm
