"""FrontEndPipeline: extraction + SearchForInitialization over a camera stream, overlapped on
several HIP streams (C ABI orb_pipeline_*, csrc/orb_pipeline.hip)."""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import FrameBounds, check, hip_lib, ptr


class FrontEndPipeline:
    """One step = ORBextractor on B frames + SearchForInitialization(F_b, F_b+1), b < B-1
    (reference Frame.cc:56-128, Tracking.cc:392-393), cut into `n_streams` overlapped chunks."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, scoreType=1, fastTh=20, device=0, max_batch=256,
                 n_streams=4):
        self._lib = hip_lib()
        h = ctypes.c_void_p()
        check(self._lib.orb_pipeline_create(int(nfeatures), float(scaleFactor), int(nlevels), int(scoreType),
                                            int(fastTh), int(device), int(max_batch), int(n_streams), ctypes.byref(h)))
        self._h = h
        self.max_keypoints = int(self._lib.orb_pipeline_max_keypoints(self._h))
        self.n_streams = int(self._lib.orb_pipeline_streams(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orb_pipeline_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def run(self, d_imgs, d_kps, d_desc, d_counts, d_matches12, d_nmatches, nnratio=0.9, checkOri=True, window=100,
            stream=None):
        """d_imgs (B, H, W) uint8; outputs as ORBextractor.extract_batch_device and
        ORBmatcher.search_for_initialization_batch_device (pairs (b, b+1))."""
        import torch

        B, h, w = d_imgs.shape
        s = stream if stream is not None else torch.cuda.current_stream(d_imgs.device)
        check(self._lib.orb_pipeline_extract_and_match(
            self._h, int(B), ptr(d_imgs), int(w), int(h), int(d_imgs.stride(1)), int(d_imgs.stride(0)), ptr(d_kps),
            ptr(d_desc), ptr(d_counts), FrameBounds(0, int(w), 0, int(h)), float(nnratio), int(bool(checkOri)),
            int(window), ptr(d_matches12), ptr(d_nmatches), ctypes.c_void_p(s.cuda_stream)))

    def run_undistorted(self, d_imgs, K, distCoef, d_kps, d_kps_un, d_desc, d_counts, d_matches12, d_nmatches,
                        nnratio=0.9, checkOri=True, window=100, stream=None):
        """The same step for a calibrated camera with distortion (Frame::Frame's
        UndistortKeyPoints, Frame.cc:69): keypoints are undistorted into d_kps_un between
        extraction and matching, and the pairs are matched on mvKeysUn inside the camera's
        ComputeImageBounds (Frame.cc:321-349).  k1 == 0 copies the records (Frame.cc:291-295)."""
        import torch

        from . import camera

        B, h, w = d_imgs.shape
        k4, d4 = camera.camera_k4(K), camera.dist4(distCoef)
        b = camera.image_bounds(int(w), int(h), k4, d4)
        s = stream if stream is not None else torch.cuda.current_stream(d_imgs.device)
        check(self._lib.orb_pipeline_extract_undistort_and_match(
            self._h, int(B), ptr(d_imgs), int(w), int(h), int(d_imgs.stride(1)), int(d_imgs.stride(0)), ptr(k4),
            ptr(d4), ptr(d_kps), ptr(d_kps_un), ptr(d_desc), ptr(d_counts), b, float(nnratio), int(bool(checkOri)),
            int(window), ptr(d_matches12), ptr(d_nmatches), ctypes.c_void_p(s.cuda_stream)))

    def profile_enable(self, enable: bool = True) -> None:
        check(self._lib.orb_pipeline_profile_enable(self._h, int(enable)))

    def profile_read(self) -> dict:
        ms = np.zeros(16, np.float64)
        n = np.zeros(16, np.int64)
        k = check(self._lib.orb_pipeline_profile_read(self._h, ptr(ms), ptr(n), 16))
        return {self._lib.orb_profile_stage_name(i).decode(): (float(ms[i]), int(n[i])) for i in range(k)}
