#!/usr/bin/env python3
"""tests/golden/kf_records_scene_320x240.{keys,des}.bin: the two oracle-extracted scene frames
of tests/golden (scene_320x240_nf500{,_f1}.npz) as two keyframes of the reference's map streams
kfKeyPoints.bin / kfDescriptors.bin, laid out by an independent struct-level restatement of
SaveLoadWorld.h:1406-1460 (header 0xEB 0x90, size_t / int count, raw fields), not by the product."""
import pathlib
import struct

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
G = ROOT / "tests" / "golden"
KP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
               ("octave", "<i4"), ("class_id", "<i4")])


def keys_record(k):
    out = bytearray(b"\xeb\x90") + struct.pack("<Q", len(k))
    for r in k:
        out += struct.pack("<5f2i", float(r["x"]), float(r["y"]), float(r["size"]), float(r["angle"]),
                           float(r["response"]), int(r["octave"]), int(r["class_id"]))
    return bytes(out)


def des_record(d):
    out = bytearray(b"\xeb\x90") + struct.pack("<i", len(d))
    for row in d:
        out += bytes(row.tolist())
    return bytes(out)


def main():
    keys, des = b"", b""
    for name in ("scene_320x240_nf500", "scene_320x240_nf500_f1"):
        z = np.load(G / f"{name}.npz")
        k = z["kps"].reshape(-1).view(KP)
        keys += keys_record(k)
        des += des_record(z["desc"])
    (G / "kf_records_scene_320x240.keys.bin").write_bytes(keys)
    (G / "kf_records_scene_320x240.des.bin").write_bytes(des)
    print(len(keys), len(des))


if __name__ == "__main__":
    main()
