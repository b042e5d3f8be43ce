"""Frame keypoint geometry: Frame::UndistortKeyPoints / ComputeImageBounds over the HIP C ABI.

Reference: src/Frame.cc:289-319 (UndistortKeyPoints: cv::undistortPoints(pts, K, mDistCoef,
noArray(), K), a plain copy when k1 == 0) and 321-349 (ComputeImageBounds); the camera as
Tracking.cc:52-70 reads it (K from fx, fy, cx, cy; mDistCoef = k1, k2, p1, p2).  The arithmetic
runs in csrc/orb_frame.hip (k_undistort); nothing here computes on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import KEYPOINT_DTYPE, FrameBounds, check, hip_lib, ptr


def camera_k4(K) -> np.ndarray:
    """(fx, fy, cx, cy) as float32 from a 3x3 camera matrix or a 4-vector."""
    K = np.asarray(K, np.float32)
    if K.shape == (3, 3):
        if K[0, 1] != 0 or K[1, 0] != 0 or K[2, 0] != 0 or K[2, 1] != 0 or K[2, 2] != 1:
            raise ValueError("K must be [fx 0 cx; 0 fy cy; 0 0 1] (Tracking.cc:52-63)")
        return np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], np.float32)
    if K.shape == (4,):
        return np.ascontiguousarray(K)
    raise ValueError("K must be 3x3 or (fx, fy, cx, cy)")


def dist4(distCoef) -> np.ndarray:
    """mDistCoef (k1, k2, p1, p2) as float32."""
    d = np.asarray(distCoef, np.float32).reshape(-1)
    if d.shape != (4,):
        raise ValueError("distCoef must hold (k1, k2, p1, p2) (Tracking.cc:65-69)")
    return np.ascontiguousarray(d)


def undistort_keypoints(kps, K, distCoef, device: int = -1) -> np.ndarray:
    """Frame::UndistortKeyPoints: mvKeys -> mvKeysUn (records copied, pt undistorted)."""
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.empty_like(kps)
    k4, d4 = camera_k4(K), dist4(distCoef)
    check(hip_lib().orb_undistort_keypoints(ptr(kps), len(kps), ptr(k4), ptr(d4), int(device), ptr(out)))
    return out


def undistort_points(xy, K, distCoef, device: int = -1) -> np.ndarray:
    """cv::undistortPoints(xy, K, distCoef, noArray(), K) for an (n, 2) float32 array."""
    xy = np.ascontiguousarray(np.asarray(xy, np.float32).reshape(-1, 2))
    out = np.empty_like(xy)
    k4, d4 = camera_k4(K), dist4(distCoef)
    check(hip_lib().orb_undistort_points(ptr(xy), len(xy), ptr(k4), ptr(d4), int(device), ptr(out)))
    return out


def compute_image_bounds(cols: int, rows: int, K, distCoef, device: int = -1) -> FrameBounds:
    """Frame::ComputeImageBounds -> (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
    b = FrameBounds()
    k4, d4 = camera_k4(K), dist4(distCoef)
    check(hip_lib().orb_compute_image_bounds(int(cols), int(rows), ptr(k4), ptr(d4), int(device), ctypes.byref(b)))
    return b


_BOUNDS = {}


def image_bounds(cols: int, rows: int, K, distCoef) -> FrameBounds:
    """The bounds Frame keeps: the reference computes them once, on the first frame, into
    static members (Frame.cc:73-86, mbInitialComputations) and every later frame of the same
    camera reuses them; here they are kept per (image size, K, distCoef), so only a new camera
    or image size costs a device round trip.  Returns a copy (callers may not mutate the cache)."""
    k4, d4 = camera_k4(K), dist4(distCoef)
    key = (int(cols), int(rows), k4.tobytes(), d4.tobytes())
    b = _BOUNDS.get(key)
    if b is None:
        b = _BOUNDS[key] = compute_image_bounds(cols, rows, k4, d4)
    return FrameBounds(b.min_x, b.max_x, b.min_y, b.max_y)


def undistort_keypoints_batch_device(d_kps, d_counts, K, distCoef, d_kps_un=None, stream=None):
    """orb_undistort_keypoints_batch_device on extractor output ((B, cap, 28) uint8 device
    tensor + (B,) int32 counts); returns d_kps_un (same shape), enqueued on `stream`."""
    import torch

    if d_kps.dim() != 3 or d_kps.shape[2] != 28 or d_kps.dtype != torch.uint8 or not d_kps.is_contiguous():
        raise TypeError("d_kps must be a contiguous (B, cap, 28) uint8 device tensor")
    B, cap = int(d_kps.shape[0]), int(d_kps.shape[1])
    if d_counts.shape != (B,) or d_counts.dtype != torch.int32 or d_counts.device != d_kps.device:
        raise TypeError("d_counts must be a (B,) int32 tensor on d_kps's device")
    if d_kps_un is None:
        d_kps_un = torch.empty_like(d_kps)
    elif d_kps_un.shape != d_kps.shape or d_kps_un.device != d_kps.device or not d_kps_un.is_contiguous():
        raise TypeError("d_kps_un must match d_kps")
    k4, d4 = camera_k4(K), dist4(distCoef)
    s = stream if stream is not None else torch.cuda.current_stream(d_kps.device)
    check(hip_lib().orb_undistort_keypoints_batch_device(ptr(d_kps), ptr(d_counts), cap, B, ptr(k4), ptr(d4),
                                                         ptr(d_kps_un), ctypes.c_void_p(s.cuda_stream)))
    return d_kps_un
