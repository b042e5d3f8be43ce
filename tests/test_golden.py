"""Committed golden fixtures (tests/golden/, made by scripts/gen_golden.py from the oracle):
the oracle must reproduce them bit-for-bit (CPU), and so must the HIP path (GPU)."""
import hashlib
import json
import pathlib

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle, search_for_initialization

G = pathlib.Path(__file__).resolve().parent / "golden"
META = json.loads((G / "golden.json").read_text())


def sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def frame(meta):
    src = meta["src"]
    if src[0] == "stream":
        return orb.synth_stream(meta["W"], meta["H"], stream=src[1], first=src[2], count=1)[0]
    return orb.synth_special(src[1], meta["W"], meta["H"], seed=src[2])


@pytest.mark.parametrize("name", sorted(META["fixtures"]))
def test_oracle_reproduces_fixture(name):
    m = META["fixtures"][name]
    img = frame(m)
    assert sha(img) == m["frame_sha256"], "synthetic generator drifted"
    k, d = Oracle(m["nfeatures"], 1.2, m["nlevels"], 1, 20).extract(img)
    g = np.load(G / f"{name}.npz")
    assert k.view(np.uint8).reshape(-1, 28).tobytes() == g["kps"].tobytes()
    assert d.tobytes() == g["desc"].tobytes()


def test_oracle_reproduces_match_fixture():
    a = np.load(G / "scene_320x240_nf500.npz")
    b = np.load(G / "scene_320x240_nf500_f1.npz")
    ka = a["kps"].view(orb.KEYPOINT_DTYPE).reshape(-1)
    kb = b["kps"].view(orb.KEYPOINT_DTYPE).reshape(-1)
    prev = np.ascontiguousarray(np.stack([ka["x"], ka["y"]], 1).astype(np.float32))
    n, m12 = search_for_initialization(ka, a["desc"], kb, b["desc"], 320, 240, prev, 0.9, True, 100)
    g = np.load(G / "match_320x240_f0_f1.npz")
    assert n == META["matches"]["match_320x240_f0_f1"]["nmatches"]
    assert np.array_equal(m12, g["m12"]) and prev.tobytes() == g["prev"].tobytes()


def test_oracle_reproduces_c1_digest():
    m = META["digests"]["c1c2_640x480_nf1000"]
    ora = Oracle(1000, 1.2, 8, 1, 20)
    f = orb.synth_stream(640, 480, stream=0, first=0, count=1)[0]
    assert sha(f) == m["frames"][0]["frame_sha256"]
    k, d = ora.extract(f)
    assert sha(k) == m["frames"][0]["kps_sha256"] and sha(d) == m["frames"][0]["desc_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(META["digests"]))
def test_gpu_matches_golden_digests(name):
    m = META["digests"][name]
    ext = orb.ORBextractor(m["nfeatures"], 1.2, m["nlevels"], orb.FAST_SCORE, 20, device=0)
    frames = orb.synth_stream(m["W"], m["H"], stream=0, first=0, count=len(m["frames"]))
    outs = []
    for f, e in zip(frames, m["frames"]):
        assert sha(f) == e["frame_sha256"]
        k, d = ext(f)
        assert len(k) == e["n"]
        assert sha(k) == e["kps_sha256"] and sha(d) == e["desc_sha256"]
        outs.append((k, d))
    F1 = orb.Frame(outs[0][0], outs[0][1], m["W"], m["H"])
    F2 = orb.Frame(outs[1][0], outs[1][1], m["W"], m["H"])
    prev = np.ascontiguousarray(np.stack([F1.mvKeys["x"], F1.mvKeys["y"]], 1).astype(np.float32))
    m12 = []
    n = orb.ORBmatcher(0.9, True).SearchForInitialization(F1, F2, prev, m12, 100)
    assert n == m["match_f0_f1"]["nmatches"]
    assert sha(np.array(m12, np.int32)) == m["match_f0_f1"]["m12_sha256"]
    assert sha(prev) == m["match_f0_f1"]["prev_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(META["fixtures"]))
def test_gpu_matches_fixture(name):
    m = META["fixtures"][name]
    ext = orb.ORBextractor(m["nfeatures"], 1.2, m["nlevels"], orb.FAST_SCORE, 20, device=0)
    k, d = ext(frame(m))
    g = np.load(G / f"{name}.npz")
    assert k.view(np.uint8).reshape(-1, 28).tobytes() == g["kps"].tobytes()
    assert (d if d is not None else np.zeros((0, 32), np.uint8)).tobytes() == g["desc"].tobytes()
