"""ctypes bindings to the in-tree native libraries.

``liborb_hip.so`` is the product (HIP kernels + the C ABI of ``include/orb_abi.h``);
``libsynth.so`` is the host-only synthetic frame generator.  Both are built in-tree by
``__graft_entry__.build()``.  There is no CPU fallback: if the HIP library is missing or
cannot be loaded, every entry point raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

import numpy as np

PKG_DIR = pathlib.Path(__file__).resolve().parent
# ORB_HIP_LIB names an experiment build of the same library (scripts/build_variant.sh)
HIP_LIB_PATH = pathlib.Path(os.environ["ORB_HIP_LIB"]) if os.environ.get("ORB_HIP_LIB") else PKG_DIR / "liborb_hip.so"
SYNTH_LIB_PATH = PKG_DIR / "libsynth.so"

# cv::KeyPoint layout (28 bytes), reference include/SaveLoadWorld.h:1406-1425
KEYPOINT_DTYPE = np.dtype(
    [
        ("x", "<f4"),
        ("y", "<f4"),
        ("size", "<f4"),
        ("angle", "<f4"),
        ("response", "<f4"),
        ("octave", "<i4"),
        ("class_id", "<i4"),
    ]
)
assert KEYPOINT_DTYPE.itemsize == 28

ORB_OK = 0
ORB_EINVAL = -22
ORB_ENOMEM = -12
ORB_ERANGE = -34
ORB_EDEVICE = -5
ORB_ENOTSUP = -95

HARRIS_SCORE = 0
FAST_SCORE = 1


class NativeLibraryError(RuntimeError):
    pass


class OrbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"orb status {code}: {msg}")
        self.code = code


class FrameBounds(ctypes.Structure):
    _fields_ = [("min_x", ctypes.c_int), ("max_x", ctypes.c_int), ("min_y", ctypes.c_int), ("max_y", ctypes.c_int)]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float

MAX_VIEW_LEVELS = 16


class FrameView(ctypes.Structure):
    """orb_frame_view_t (include/orb_abi.h): a Frame / KeyFrame as the matchers see it."""

    _fields_ = [
        ("kps", _vp),
        ("desc", _vp),
        ("n", ctypes.c_int32),
        ("nlevels", ctypes.c_int32),
        ("bounds", FrameBounds),
        ("scale_factors", _f * MAX_VIEW_LEVELS),
        ("level_sigma2", _f * MAX_VIEW_LEVELS),
        ("fx", _f),
        ("fy", _f),
        ("cx", _f),
        ("cy", _f),
        ("Rcw", _f * 9),
        ("tcw", _f * 3),
        ("Ow", _f * 3),
    ]


class MapPoints(ctypes.Structure):
    """orb_map_points_t: MapPoint attributes read by the projection matchers."""

    _fields_ = [("pos", _vp), ("normal", _vp), ("dmin", _vp), ("dmax", _vp), ("desc", _vp), ("n", ctypes.c_int32)]


class FeatureVectorCSR(ctypes.Structure):
    """orb_feature_vector_t: DBoW2::FeatureVector as CSR (nodes, offsets, features)."""

    _fields_ = [("nodes", _vp), ("offsets", _vp), ("features", _vp), ("n_nodes", ctypes.c_int32)]


_pv = ctypes.POINTER(FrameView)
_pi = ctypes.POINTER(_i)

# name -> (restype, argtypes); every symbol declared in include/orb_abi.h
HIP_SIGNATURES = {
    "orb_last_error": (ctypes.c_char_p, []),
    "orb_version": (ctypes.c_char_p, []),
    "orb_extractor_create": (_i, [_i, _f, _i, _i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "orb_extractor_destroy": (_i, [_vp]),
    "orb_get_levels": (_i, [_vp]),
    "orb_get_scale_factor": (_f, [_vp]),
    "orb_get_max_keypoints": (_i, [_vp]),
    "orb_get_level_info": (_i, [_vp, _vp, _vp]),
    "orb_extract": (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _vp, ctypes.POINTER(_i)]),
    "orb_extract_batch_device": (_i, [_vp, _i, _vp, _i, _i, _i, _i64, _vp, _vp, _vp, _vp]),
    "orb_extract_batch": (_i, [_vp, _i, _vp, _i, _i, _i, _i64, _vp, _vp, _vp]),
    "orb_extract_batch_device_color": (_i, [_vp, _i, _vp, _i, _i, _i, _i64, _i, _i, _vp, _vp, _vp, _vp]),
    "orb_extract_color": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp, ctypes.POINTER(_i)]),
    "orb_descriptor_distance": (_i, [_vp, _vp]),
    "orb_search_for_initialization": (
        _i,
        [_vp, _vp, _i, _vp, _vp, _i, FrameBounds, _f, _i, _i, _vp, _vp, ctypes.POINTER(_i)],
    ),
    "orb_search_for_initialization_batch_device": (
        _i,
        [_vp, _vp, _vp, _i, _i, _vp, _vp, FrameBounds, _f, _i, _i, _vp, _vp, _vp, _vp],
    ),
    "orb_match_release_stream_scratch": (_i, [_vp]),
    "orb_stream_create_dedicated": (_i, [ctypes.POINTER(_vp)]),
    "orb_debug_set_fast_corner_list": (_i, [_vp, _i]),
    "orb_search_by_bow_batch_device": (_i, [_i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _f, _i, _vp,
                                            _vp, _vp]),
    "orb_stream_destroy": (_i, [_vp]),
    "orb_features_in_area": (_i, [_pv, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i]),
    "orb_frame_is_in_frustum": (_i, [_pv, MapPoints, _f, _vp, _vp, _vp, _vp, _vp, _i]),
    "orb_search_by_bow_kf_f": (_i, [_pv, _vp, FeatureVectorCSR, _pv, FeatureVectorCSR, _f, _i, _vp, _pi, _i]),
    "orb_search_by_bow_kf_kf": (_i, [_pv, _vp, FeatureVectorCSR, _pv, _vp, FeatureVectorCSR, _f, _i, _vp, _pi, _i]),
    "orb_search_for_triangulation": (
        _i,
        [_pv, _vp, FeatureVectorCSR, _pv, _vp, FeatureVectorCSR, _vp, _f, _i, _vp, _pi, _i],
    ),
    "orb_window_search": (_i, [_pv, _vp, _pv, _i, _i, _i, _f, _i, _vp, _pi, _i]),
    "orb_search_by_projection_local": (_i, [_pv, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _vp, _pi, _i]),
    "orb_search_by_projection_f2f": (_i, [_pv, MapPoints, _vp, _pv, _vp, _i, _f, _vp, _pi, _i]),
    "orb_search_by_projection_motion": (_i, [_pv, _vp, _pv, MapPoints, _vp, _f, _i, _vp, _pi, _i]),
    "orb_search_by_projection_reloc": (_i, [_pv, _vp, _pv, MapPoints, _vp, _f, _i, _i, _vp, _pi, _i]),
    "orb_search_by_projection_sim3": (_i, [_pv, _vp, MapPoints, _vp, _i, _vp, _pi, _i]),
    "orb_search_by_sim3": (_i, [_pv, MapPoints, _vp, _pv, MapPoints, _vp, _vp, _vp, _vp, _vp, _f, _vp, _pi, _i]),
    "orb_fuse": (_i, [_pv, MapPoints, _vp, _f, _i, _vp, _pi, _i]),
    "orb_pipeline_create": (_i, [_i, _f, _i, _i, _i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "orb_pipeline_destroy": (_i, [_vp]),
    "orb_pipeline_max_keypoints": (_i, [_vp]),
    "orb_pipeline_streams": (_i, [_vp]),
    "orb_pipeline_extract_and_match": (
        _i,
        [_vp, _i, _vp, _i, _i, _i, _i64, _vp, _vp, _vp, FrameBounds, _f, _i, _i, _vp, _vp, _vp],
    ),
    "orb_pipeline_extract_undistort_and_match": (
        _i,
        [_vp, _i, _vp, _i, _i, _i, _i64, _vp, _vp, _vp, _vp, _vp, _vp, FrameBounds, _f, _i, _i, _vp, _vp, _vp],
    ),
    "orb_undistort_keypoints_batch_device": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp]),
    "orb_undistort_keypoints": (_i, [_vp, _i, _vp, _vp, _i, _vp]),
    "orb_undistort_points": (_i, [_vp, _i, _vp, _vp, _i, _vp]),
    "orb_compute_image_bounds": (_i, [_i, _i, _vp, _vp, _i, ctypes.POINTER(FrameBounds)]),
    "orb_pipeline_profile_enable": (_i, [_vp, _i]),
    "orb_pipeline_profile_read": (_i, [_vp, _vp, _vp, _i]),
    "orb_compute_distinctive_descriptors": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _i]),
    "orb_compute_distinctive_descriptors_device": (_i, [_i, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "orb_keypoint_record_bytes": (ctypes.c_size_t, [ctypes.c_size_t]),
    "orb_descriptor_record_bytes": (ctypes.c_size_t, [_i]),
    "orb_write_keypoint_record": (_i, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "orb_read_keypoint_record": (_i, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_i)]),
    "orb_write_descriptor_record": (_i, [_vp, _i, _vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "orb_read_descriptor_record": (_i, [_vp, ctypes.c_size_t, _vp, _i, ctypes.POINTER(_i),
                                        ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_i)]),
    "orb_pack_keyframe_records_device": (_i, [_vp, _vp, _vp, _i, _i, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp,
                                              _vp, _vp]),
    "orb_vocabulary_load_text": (_i, [ctypes.c_char_p, _i, ctypes.POINTER(_vp)]),
    "orb_vocabulary_create": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, ctypes.POINTER(_vp)]),
    "orb_vocabulary_destroy": (_i, [_vp]),
    "orb_vocabulary_info": (_i, [_vp, _vp]),
    "orb_vocabulary_transform_features_device": (_i, [_vp, _i, _vp, _i, _vp, _vp, _vp, _vp]),
    "orb_vocabulary_transform_batch_device": (
        _i,
        [_vp, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    ),
    "orb_vocabulary_transform": (_i, [_vp, _vp, _i, _i, _vp, _vp, _pi, _vp, _vp, _vp, _pi]),
    "orb_profile_enable": (_i, [_vp, _i]),
    "orb_profile_enable_stages": (_i, [_vp, ctypes.c_uint]),
    "orb_extract_set_phases": (_i, [_vp, ctypes.c_uint]),
    "orb_profile_read": (_i, [_vp, _vp, _vp, _i]),
    "orb_profile_stage_name": (ctypes.c_char_p, [_i]),
    "orb_debug_nth_element_u32": (_i, [_vp, _i, _i]),
    "orb_debug_nth_element_wave_u32": (_i, [_vp, _i, _i, _i]),
    "orb_debug_level_image": (_i, [_vp, _i, _i, _vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "orb_debug_cell_counts": (_i, [_vp, _i, _i, _vp, _i]),
    "orb_debug_blur_image": (_i, [_vp, _i, _i, _vp]),
    "orb_debug_set_pyramid_path": (_i, [_vp, _i]),
    "orb_debug_pyramid_plan": (_i, [_vp, _pi, _pi, _pi]),
}

_hip = None
_synth = None


def _bind_torch_runtime() -> None:
    """Import torch before dlopen-ing liborb_hip.so.

    PyTorch-ROCm ships its own libamdhip64 (same SONAME, libamdhip64.so.7).  Loading it
    first makes the dynamic linker bind liborb_hip.so to that copy, so the process has ONE
    HIP runtime and torch-allocated device memory / streams are valid in our kernels.  (If
    liborb_hip.so were loaded first, torch would start a second runtime and see no GPU.)
    """
    try:
        import torch  # noqa: F401
    except Exception:  # torch absent: the C ABI works standalone on /opt/rocm's runtime
        pass


def hip_lib() -> ctypes.CDLL:
    """Load liborb_hip.so (fails loudly: there is no CPU fallback)."""
    global _hip
    if _hip is None:
        _bind_torch_runtime()
        if not HIP_LIB_PATH.exists():
            raise NativeLibraryError(
                f"{HIP_LIB_PATH} is missing; run `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        try:
            lib = ctypes.CDLL(str(HIP_LIB_PATH), mode=os.RTLD_LOCAL)
        except OSError as e:  # pragma: no cover - environment dependent
            raise NativeLibraryError(f"cannot load {HIP_LIB_PATH}: {e}") from e
        for name, (res, args) in HIP_SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                if os.environ.get("ORB_HIP_LIB"):  # an experiment build of an older ABI
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        _hip = lib
    return _hip


def synth_lib() -> ctypes.CDLL:
    global _synth
    if _synth is None:
        if not SYNTH_LIB_PATH.exists():
            raise NativeLibraryError(f"{SYNTH_LIB_PATH} is missing; run __graft_entry__.build()")
        lib = ctypes.CDLL(str(SYNTH_LIB_PATH))
        lib.orb_synth_stream.restype = _i
        lib.orb_synth_stream.argtypes = [_i, _i, ctypes.c_uint64, ctypes.c_uint64, _i, _vp, _i, _i64]
        lib.orb_synth_special.restype = _i
        lib.orb_synth_special.argtypes = [_i, _i, _i, ctypes.c_uint64, _vp, _i]
        _synth = lib
    return _synth


def check(code: int) -> int:
    if code < 0:
        msg = hip_lib().orb_last_error()
        raise OrbError(code, msg.decode() if msg else "")
    return code


def ptr(a) -> ctypes.c_void_p:
    """Data pointer of a numpy array or torch tensor."""
    if a is None:
        return ctypes.c_void_p(0)
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    return ctypes.c_void_p(a.data_ptr())
