"""ORBextractor — host mirror of the reference class over the HIP C ABI.

Reference: include/ORBextractor.h:30-80, src/ORBextractor.cc:457-822.  Same constructor
arguments and defaults, same ``operator()`` semantics (``__call__`` here):

* an empty image returns without producing outputs (ORBextractor.cc:721-722) — here
  ``(None, None)``;
* a non-empty image yields N <= nfeatures keypoints (cv::KeyPoint records,
  ``KEYPOINT_DTYPE``) and an N x 32 uint8 descriptor matrix, or ``None`` descriptors when
  N == 0 (``_descriptors.release()``, ORBextractor.cc:738-739);
* the mask argument is accepted and ignored, as the reference's FAST ignores it.

All arithmetic runs in the HIP kernels of csrc/orb_hip.hip; this module only marshals.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import FAST_SCORE, HARRIS_SCORE, KEYPOINT_DTYPE, check, hip_lib, ptr


class ORBextractor:
    HARRIS_SCORE = HARRIS_SCORE
    FAST_SCORE = FAST_SCORE

    def __init__(
        self,
        nfeatures: int = 1000,
        scaleFactor: float = 1.2,
        nlevels: int = 8,
        scoreType: int = FAST_SCORE,
        fastTh: int = 20,
        device: int = 0,
        max_batch: int = 1,
    ):
        self._lib = hip_lib()
        h = ctypes.c_void_p()
        check(self._lib.orb_extractor_create(nfeatures, scaleFactor, nlevels, scoreType, fastTh, device, max_batch,
                                             ctypes.byref(h)))
        self._h = h
        self.nfeatures = nfeatures
        self.nlevels = nlevels
        self.scoreType = scoreType
        self.fastTh = fastTh
        self.device = device
        self.max_batch = max_batch
        self.max_keypoints = check(self._lib.orb_get_max_keypoints(self._h))
        fpl = np.zeros(nlevels, np.int32)
        sf = np.zeros(nlevels, np.float32)
        check(self._lib.orb_get_level_info(self._h, ptr(fpl), ptr(sf)))
        self.mnFeaturesPerLevel = fpl
        self.mvScaleFactor = sf

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.orb_extractor_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # ORBextractor::GetLevels / GetScaleFactor (ORBextractor.h:47-51)
    def GetLevels(self) -> int:
        return self._lib.orb_get_levels(self._h)

    def GetScaleFactor(self) -> float:
        return float(self._lib.orb_get_scale_factor(self._h))

    def __call__(self, image, mask=None):
        img = np.asarray(image)
        if img.size == 0:
            return None, None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise TypeError("image must be a 2-D uint8 array (CV_8UC1), ORBextractor.cc:725")
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = self.max_keypoints
        kps = np.empty(cap, KEYPOINT_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        n = ctypes.c_int()
        check(self._lib.orb_extract(self._h, ptr(img), w, h, img.strides[0], ptr(kps), cap, ptr(desc), ctypes.byref(n)))
        n = n.value
        return kps[:n].copy(), (desc[:n].copy() if n > 0 else None)

    def extract_batch(self, images: np.ndarray):
        """B host frames (B, H, W) uint8 -> list of (keypoints, descriptors)."""
        imgs = np.ascontiguousarray(images, dtype=np.uint8)
        B, h, w = imgs.shape
        cap = self.max_keypoints
        kps = np.empty((B, cap), KEYPOINT_DTYPE)
        desc = np.empty((B, cap, 32), np.uint8)
        counts = np.zeros(B, np.int32)
        check(self._lib.orb_extract_batch(self._h, B, ptr(imgs), w, h, w, w * h, ptr(kps), ptr(desc), ptr(counts)))
        return [(kps[b, : counts[b]].copy(), desc[b, : counts[b]].copy() if counts[b] else None) for b in range(B)]

    def extract_batch_device(self, d_imgs, d_kps=None, d_desc=None, d_counts=None, stream=None):
        """Device-resident batch: d_imgs is a (B, H, W) uint8 torch tensor on this device.

        Returns (d_kps (B, cap, 28) uint8, d_desc (B, cap, 32) uint8, d_counts (B,) int32),
        enqueued on `stream` (a torch.cuda.Stream; default: the current stream).
        """
        import torch

        if d_imgs.dim() != 3:
            raise TypeError("d_imgs must be a (B, H, W) uint8 device tensor")
        B, h, w = d_imgs.shape
        d_kps, d_desc, d_counts = self._device_io(d_imgs, 1, d_kps, d_desc, d_counts)
        s = stream if stream is not None else torch.cuda.current_stream(d_imgs.device)
        check(self._lib.orb_extract_batch_device(self._h, B, ptr(d_imgs), w, h, d_imgs.stride(1), d_imgs.stride(0),
                                                 ptr(d_kps), ptr(d_desc), ptr(d_counts),
                                                 ctypes.c_void_p(s.cuda_stream)))
        return d_kps, d_desc, d_counts


    def _device_io(self, d_imgs, cn, d_kps, d_desc, d_counts):
        """Validate a device batch (the C ABI takes raw pointers: a wrong tensor would be
        silent garbage or out-of-bounds device writes) and allocate missing outputs."""
        import torch

        B = d_imgs.shape[0]
        dev = d_imgs.device
        if dev.type != "cuda" or (dev.index if dev.index is not None else torch.cuda.current_device()) != self.device:
            raise ValueError(f"d_imgs is on {dev}, the extractor on cuda:{self.device}")
        if d_imgs.dtype != torch.uint8:
            raise TypeError("d_imgs must be uint8")
        if B > self.max_batch:
            raise ValueError(f"batch {B} exceeds max_batch {self.max_batch}")
        # pixels of a row contiguous (row pitch = stride(1), frame pitch = stride(0))
        if (cn == 1 and d_imgs.stride(2) != 1) or (cn > 1 and (d_imgs.stride(3) != 1 or d_imgs.stride(2) != cn)):
            raise ValueError("image rows must be contiguous")
        cap = self.max_keypoints
        outs = []
        for t, shape in ((d_kps, (B, cap, 28)), (d_desc, (B, cap, 32)), (d_counts, (B,))):
            dt = torch.int32 if len(shape) == 1 else torch.uint8
            if t is None:
                t = torch.empty(shape, dtype=dt, device=dev)
            elif (t.device != dev or t.dtype != dt or not t.is_contiguous() or t.dim() != len(shape)
                  or tuple(t.shape[1:]) != shape[1:] or t.shape[0] < B):
                raise ValueError(f"output tensor must be a contiguous {dt} tensor of shape {shape} (or more "
                                 f"frames) on {dev}")
            outs.append(t)
        return outs

    # ---- colour frames: Tracking::GrabImage's cvtColor fused with level 0 (Tracking.cc:202-207)
    def extract_color(self, image, rgb: bool = True):
        """operator() on cvtColor(image, mbRGB ? CV_RGB2GRAY : CV_BGR2GRAY); image (H, W, 3|4) uint8."""
        img = np.asarray(image)
        if img.size == 0:
            return None, None
        if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] not in (3, 4):
            raise TypeError("image must be an (H, W, 3|4) uint8 array")
        img = np.ascontiguousarray(img)
        h, w, cn = img.shape
        cap = self.max_keypoints
        kps = np.empty(cap, KEYPOINT_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        n = ctypes.c_int()
        check(self._lib.orb_extract_color(self._h, ptr(img), w, h, w * cn, cn, int(bool(rgb)), ptr(kps), cap, ptr(desc),
                                          ctypes.byref(n)))
        n = n.value
        return kps[:n].copy(), (desc[:n].copy() if n > 0 else None)

    def extract_batch_device_color(self, d_imgs, rgb: bool = True, d_kps=None, d_desc=None, d_counts=None,
                                   stream=None):
        """extract_batch_device on (B, H, W, 3|4) uint8 device frames, converted to gray on the fly."""
        import torch

        if d_imgs.dim() != 4:
            raise TypeError("d_imgs must be a (B, H, W, 3|4) uint8 device tensor")
        B, h, w, cn = d_imgs.shape
        d_kps, d_desc, d_counts = self._device_io(d_imgs, cn, d_kps, d_desc, d_counts)
        s = stream if stream is not None else torch.cuda.current_stream(d_imgs.device)
        check(self._lib.orb_extract_batch_device_color(self._h, B, ptr(d_imgs), w, h, d_imgs.stride(1),
                                                       d_imgs.stride(0), cn, int(bool(rgb)), ptr(d_kps), ptr(d_desc),
                                                       ptr(d_counts), ctypes.c_void_p(s.cuda_stream)))
        return d_kps, d_desc, d_counts

    # ---- measurement ----------------------------------------------------------------------
    def set_phases(self, mask: int) -> None:
        """Run only part of extract_batch_device (not the other entry points) on the next
        calls: 1 = pyramid, 2 = detection through descriptors (reads the pyramid phase 1 left),
        3 = both (default)."""
        check(self._lib.orb_extract_set_phases(self._h, int(mask)))

    def profile_enable(self, enable: bool = True) -> None:
        """Record a HIP-event pair around every kernel stage of extract_batch_device."""
        check(self._lib.orb_profile_enable(self._h, int(enable)))

    def profile_enable_stages(self, stages) -> None:
        """Record event pairs around the named stages only (each pair is a stream boundary)."""
        names = [self._lib.orb_profile_stage_name(i).decode() for i in range(16)]
        mask = 0
        for s in stages:
            mask |= 1 << names.index(s)
        check(self._lib.orb_profile_enable_stages(self._h, mask))

    def profile_read(self) -> dict:
        """{stage_name: (cumulative_ms, launches)} since profile_enable (synchronises)."""
        ms = np.zeros(16, np.float64)
        n = np.zeros(16, np.int64)
        k = check(self._lib.orb_profile_read(self._h, ptr(ms), ptr(n), 16))
        return {self._lib.orb_profile_stage_name(i).decode(): (float(ms[i]), int(n[i])) for i in range(k)}


def keypoints_from_bytes(raw: np.ndarray, n: int) -> np.ndarray:
    """View n records of a (cap, 28) uint8 buffer as KEYPOINT_DTYPE."""
    return np.ascontiguousarray(raw[:n]).view(KEYPOINT_DTYPE).reshape(-1)
