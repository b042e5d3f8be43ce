#!/usr/bin/env python3
"""Regenerate tests/golden/ from the CPU oracle (oracle/liborb_oracle.so).

The reference has no tests or fixtures, so the goldens are the oracle's
outputs on deterministic synthetic frames (csrc/synth.c).  They pin the oracle against
regressions and give the GPU tests a target that does not need the oracle at run time:
  - small fixtures (npz of raw bytes): keypoints, descriptors, matches;
  - SHA-256 digests for the BASELINE.json configs at full size.
"""
import hashlib
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orbslam_jpminipc_amd as orb  # noqa: E402
from oracle_lib import Oracle, search_for_initialization  # noqa: E402

OUT = ROOT / "tests" / "golden"

FIXTURES = [
    # name, W, H, nfeatures, nlevels, frame source
    ("scene_320x240_nf500", 320, 240, 500, 8, ("stream", 0, 0)),
    ("scene_320x240_nf500_f1", 320, 240, 500, 8, ("stream", 0, 1)),
    ("lowtex_320x240_nf500", 320, 240, 500, 8, ("special", orb.SYN_LOWTEX, 2)),
    ("noise_160x120_nf300", 160, 120, 300, 4, ("special", orb.SYN_NOISE, 3)),
]
DIGESTS = [
    ("c1c2_640x480_nf1000", 640, 480, 1000, 8, 3),
    ("init_640x480_nf2000", 640, 480, 2000, 8, 2),
    ("c4_1241x376_nf2000", 1241, 376, 2000, 8, 2),
    ("c5_1280x720_nf2500", 1280, 720, 2500, 8, 2),
]


def frame(W, H, src):
    if src[0] == "stream":
        return orb.synth_stream(W, H, stream=src[1], first=src[2], count=1)[0]
    return orb.synth_special(src[1], W, H, seed=src[2])


def sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    meta = {"fixtures": {}, "digests": {}, "matches": {}}
    for name, W, H, nf, nl, src in FIXTURES:
        img = frame(W, H, src)
        k, d = Oracle(nf, 1.2, nl, 1, 20).extract(img)
        np.savez_compressed(OUT / f"{name}.npz", kps=k.view(np.uint8).reshape(-1, 28), desc=d)
        meta["fixtures"][name] = {"W": W, "H": H, "nfeatures": nf, "nlevels": nl, "src": list(src),
                                  "frame_sha256": sha(img), "n": int(len(k))}
    # a match fixture between the two scene frames
    a = np.load(OUT / "scene_320x240_nf500.npz")
    b = np.load(OUT / "scene_320x240_nf500_f1.npz")
    ka, kb = a["kps"].view(orb.KEYPOINT_DTYPE).reshape(-1), b["kps"].view(orb.KEYPOINT_DTYPE).reshape(-1)
    prev = np.ascontiguousarray(np.stack([ka["x"], ka["y"]], 1).astype(np.float32))
    n, m12 = search_for_initialization(ka, a["desc"], kb, b["desc"], 320, 240, prev, 0.9, True, 100)
    np.savez_compressed(OUT / "match_320x240_f0_f1.npz", m12=m12, prev=prev)
    meta["matches"]["match_320x240_f0_f1"] = {"nmatches": int(n), "nnratio": 0.9, "checkOri": True, "window": 100}
    for name, W, H, nf, nl, nframes in DIGESTS:
        ora = Oracle(nf, 1.2, nl, 1, 20)
        frames = orb.synth_stream(W, H, stream=0, first=0, count=nframes)
        ent = []
        outs = []
        for f in frames:
            k, d = ora.extract(f)
            outs.append((k, d))
            ent.append({"frame_sha256": sha(f), "n": int(len(k)), "kps_sha256": sha(k), "desc_sha256": sha(d)})
        k0, d0 = outs[0]
        k1, d1 = outs[1]
        prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1).astype(np.float32))
        n, m12 = search_for_initialization(k0, d0, k1, d1, W, H, prev, 0.9, True, 100)
        meta["digests"][name] = {"W": W, "H": H, "nfeatures": nf, "nlevels": nl, "frames": ent,
                                 "match_f0_f1": {"nmatches": int(n), "m12_sha256": sha(m12),
                                                 "prev_sha256": sha(prev)}}
    (OUT / "golden.json").write_text(json.dumps(meta, indent=1) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
