"""MI355X-native ORB-SLAM front end: ORBextractor + ORBmatcher over hand-written HIP kernels.

A drop-in for caomw/ORBSLAM_jpMiniPC's per-frame feature front end (ORBextractor's
FAST-on-pyramid + rBRIEF, ORBmatcher's Hamming window matching).  The product is the C ABI
in include/orb_abi.h (liborb_hip.so); this package mirrors the reference's class API on top.
"""
from ._native import (
    FAST_SCORE,
    HARRIS_SCORE,
    KEYPOINT_DTYPE,
    NativeLibraryError,
    OrbError,
    hip_lib,
)
from .extractor import ORBextractor, keypoints_from_bytes
from .matcher import Frame, ORBmatcher
from .synth import SYN_FLAT, SYN_LOWTEX, SYN_NOISE, SYN_SCENE, synth_special, synth_stream
from .vocabulary import ORBVocabulary

__all__ = [
    "ORBextractor",
    "ORBmatcher",
    "ORBVocabulary",
    "Frame",
    "KEYPOINT_DTYPE",
    "FAST_SCORE",
    "HARRIS_SCORE",
    "NativeLibraryError",
    "OrbError",
    "hip_lib",
    "keypoints_from_bytes",
    "synth_stream",
    "synth_special",
    "SYN_SCENE",
    "SYN_FLAT",
    "SYN_LOWTEX",
    "SYN_NOISE",
]
