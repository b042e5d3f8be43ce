"""Deterministic synthetic frames (see csrc/synth.c and SURVEY.md §8d)."""
from __future__ import annotations

import numpy as np

from ._native import check, ptr, synth_lib

SYN_SCENE, SYN_FLAT, SYN_LOWTEX, SYN_NOISE = 0, 1, 2, 3


def synth_stream(width: int, height: int, stream: int = 0, first: int = 0, count: int = 1) -> np.ndarray:
    """Frames [first, first+count) of a stream as a (count, height, width) uint8 array.

    Consecutive frames are crops of one scene shifted by (dx, dy) in [-6, 6]^2 plus fresh
    noise, so frame pairs (t, t+1) match under SearchForInitialization's window of 100.
    """
    out = np.empty((count, height, width), np.uint8)
    rc = synth_lib().orb_synth_stream(width, height, stream, first, count, ptr(out), width, width * height)
    if rc != 0:
        raise ValueError(f"orb_synth_stream failed ({rc})")
    return out


def synth_special(kind: int, width: int, height: int, seed: int = 0) -> np.ndarray:
    """Edge-case frame: SYN_FLAT (no corners), SYN_LOWTEX (th=7 fallback), SYN_NOISE (ties)."""
    out = np.empty((height, width), np.uint8)
    rc = synth_lib().orb_synth_special(kind, width, height, seed, ptr(out), width)
    if rc != 0:
        raise ValueError(f"orb_synth_special failed ({rc})")
    return out


__all__ = ["synth_stream", "synth_special", "SYN_SCENE", "SYN_FLAT", "SYN_LOWTEX", "SYN_NOISE", "check"]
