"""Keyframe feature records of the reference's map files (include/SaveLoadWorld.h).

SaveWorldToFile (SaveLoadWorld.h:1254) appends, per keyframe, one record to each of
``kfKeyPoints.bin`` / ``kfKeyPointsUn.bin`` (SaveLoadWorld.h:1406-1443)::

    0xEB 0x90 | size_t nKeys | nKeys x (x, y, size, angle, response: f32; octave, class_id: i32)

and to ``kfDescriptors.bin`` (SaveLoadWorld.h:1446-1460)::

    0xEB 0x90 | int nDes | nDes x 32 bytes

and LoadWroldFromFile reads them back in the same order (SaveLoadWorld.h:2098-2189), reporting
a wrong header and carrying on.  The byte work runs in liborb_hip.so (csrc/orb_persist.hip):
host writers / readers, and a device packer that turns a batch of extractor output into both
streams without a host round trip per keyframe.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from ._native import KEYPOINT_DTYPE, check, hip_lib, ptr


def keypoint_record_bytes(n: int) -> int:
    return int(hip_lib().orb_keypoint_record_bytes(n))


def descriptor_record_bytes(n: int) -> int:
    return int(hip_lib().orb_descriptor_record_bytes(n))


def write_keypoint_record(kps) -> bytes:
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.empty(keypoint_record_bytes(len(k)), np.uint8)
    w = ctypes.c_size_t()
    check(hip_lib().orb_write_keypoint_record(ptr(k), len(k), ptr(out), out.size, ctypes.byref(w)))
    return out[: w.value].tobytes()


def write_descriptor_record(desc) -> bytes:
    d = np.ascontiguousarray(np.asarray(desc, np.uint8).reshape(-1, 32))
    out = np.empty(descriptor_record_bytes(len(d)), np.uint8)
    w = ctypes.c_size_t()
    check(hip_lib().orb_write_descriptor_record(ptr(d), len(d), ptr(out), out.size, ctypes.byref(w)))
    return out[: w.value].tobytes()


def _buf(data, offset):
    b = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data.view(np.uint8).reshape(-1)
    return b[offset:]


def read_keypoint_record(data, offset: int = 0):
    """-> (keypoints, bytes consumed, header_ok) of the record at `offset`."""
    b = np.ascontiguousarray(_buf(data, offset))
    n, used, ok = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_int()
    L = hip_lib()
    # the record's own count (u64 after the 2-byte header), bounded by what the buffer can hold:
    # the output is sized to this record, not to the rest of the stream
    cap = min(struct.unpack_from("<Q", b, 2)[0], (b.size - 10) // 28) if b.size >= 10 else 0
    k = np.empty(max(cap, 1), KEYPOINT_DTYPE)
    check(L.orb_read_keypoint_record(ptr(b), b.size, ptr(k), cap, ctypes.byref(n), ctypes.byref(used),
                                     ctypes.byref(ok)))
    return k[: n.value].copy(), used.value, bool(ok.value)


def read_descriptor_record(data, offset: int = 0):
    """-> (descriptors (n, 32) uint8, bytes consumed, header_ok) of the record at `offset`."""
    b = np.ascontiguousarray(_buf(data, offset))
    cap = max(min(struct.unpack_from("<i", b, 2)[0], (b.size - 6) // 32), 0) if b.size >= 6 else 0
    d = np.empty((max(cap, 1), 32), np.uint8)
    n, used, ok = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_int()
    check(hip_lib().orb_read_descriptor_record(ptr(b), b.size, ptr(d), cap, ctypes.byref(n), ctypes.byref(used),
                                               ctypes.byref(ok)))
    return d[: n.value].copy(), used.value, bool(ok.value)


def read_keypoint_stream(data):
    """Every record of a kfKeyPoints.bin stream -> list of (keypoints, header_ok)."""
    out, off, size = [], 0, len(data)
    while off < size:
        k, used, ok = read_keypoint_record(data, off)
        out.append((k, ok))
        off += used
    return out


def read_descriptor_stream(data):
    """Every record of a kfDescriptors.bin stream -> list of (descriptors, header_ok)."""
    out, off, size = [], 0, len(data)
    while off < size:
        d, used, ok = read_descriptor_record(data, off)
        out.append((d, ok))
        off += used
    return out


def save_keyframe_streams(keys_path, des_path, keyframes, keys_un_path=None):
    """Append-order streams of SaveWorldToFile for [(keypoints, descriptors), ...]; with zero
    distortion mvKeysUn == mvKeys (Frame.cc:291-295), so kfKeyPointsUn.bin repeats the keys."""
    kb = b"".join(write_keypoint_record(k) for k, _ in keyframes)
    db = b"".join(write_descriptor_record(np.zeros((0, 32), np.uint8) if d is None else d) for _, d in keyframes)
    with open(keys_path, "wb") as f:
        f.write(kb)
    if keys_un_path is not None:
        with open(keys_un_path, "wb") as f:
            f.write(kb)
    with open(des_path, "wb") as f:
        f.write(db)


def pack_keyframe_records_device(d_kps, d_desc, d_counts, stream=None):
    """Device batch (orb_extract_batch_device layout) -> (keys_stream, des_stream, key_offsets,
    des_offsets) uint8 / int64 device tensors; stream lengths are offsets[B]."""
    import torch

    B, cap = int(d_kps.shape[0]), int(d_kps.shape[1])
    dev = d_kps.device
    kcap = B * keypoint_record_bytes(cap)
    dcap = B * descriptor_record_bytes(cap)
    keys = torch.empty(kcap + (kcap & 1), dtype=torch.uint8, device=dev)
    des = torch.empty(dcap + (dcap & 1), dtype=torch.uint8, device=dev)
    ko = torch.empty(B + 1, dtype=torch.int64, device=dev)
    do = torch.empty(B + 1, dtype=torch.int64, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    check(hip_lib().orb_pack_keyframe_records_device(ptr(d_kps), ptr(d_desc), ptr(d_counts), cap, B, ptr(keys),
                                                     keys.numel(), ptr(des), des.numel(), ptr(ko), ptr(do),
                                                     ctypes.c_void_p(s.cuda_stream)))
    return keys, des, ko, do
