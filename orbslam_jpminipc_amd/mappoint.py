"""MapPoint-level helpers over the C ABI (csrc/orb_mappoint.hip)."""
from __future__ import annotations

import numpy as np

from ._native import check, hip_lib, ptr


def compute_distinctive_descriptors(offsets, desc, usable=None, current=None, device: int = 0):
    """MapPoint::ComputeDistinctiveDescriptors (reference src/MapPoint.cc:185-250) for many points.

    offsets (M + 1,): point m observes rows offsets[m] .. offsets[m+1]-1 of desc (R, 32), in
    the order of its observations map; usable (R,) = keyframe not bad (None = all); current
    (M, 32) = the points' descriptors before the call (kept where no row is usable).
    Returns (best_row (M,) int32, -1 = unchanged; descriptors (M, 32) uint8).
    """
    off = np.ascontiguousarray(np.asarray(offsets, np.int32))
    d = np.ascontiguousarray(np.asarray(desc, np.uint8).reshape(-1, 32))
    M = len(off) - 1
    u = None if usable is None else np.ascontiguousarray(np.asarray(usable, np.uint8).reshape(-1))
    if u is not None and len(u) != len(d):
        raise ValueError("usable must have one flag per row")
    out = (np.zeros((max(M, 1), 32), np.uint8) if current is None
           else np.ascontiguousarray(np.array(current, np.uint8).reshape(-1, 32)))
    best = np.full(max(M, 1), -1, np.int32)
    check(hip_lib().orb_compute_distinctive_descriptors(M, ptr(off), ptr(d), ptr(u), ptr(best), ptr(out), device))
    return best[:M], out[:M]
