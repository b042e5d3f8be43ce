"""The DBoW2 vocabulary oracle (oracle/orb_oracle_voc.cpp) on the CPU: against a second,
pure-Python restatement (tests/vocab_util.py), a hand-computed known answer, and the text
format round trip; plus host-side validation of the product's vocabulary ABI."""
import ctypes

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd import _native
from orbslam_jpminipc_amd.vocabulary import write_text
from oracle_lib import Oracle
from vocab_util import OracleVocabulary, PyVocabulary, build_vocabulary, random_vocabulary

WEIGHTING_SCORING = [(0, 0), (1, 0), (2, 0), (3, 0), (0, 1), (1, 5), (2, 5), (0, 2)]


def _descs(n_frames=2, W=320, H=240, nf=500, stream=30):
    ora = Oracle(nf, 1.2, 8, 1, 20)
    return [ora.extract(f)[1] for f in orb.synth_stream(W, H, stream=stream, first=0, count=n_frames)]


def _check_same(ov, pv, d, levelsup):
    bw, bv, fn, fo, ff = ov.transform(d, levelsup)
    pbow, pfv = pv.transform(d, levelsup)
    assert bw.tolist() == list(pbow.keys())
    assert bv.view(np.uint64).tolist() == np.array(list(pbow.values()), np.float64).view(np.uint64).tolist()
    assert fn.tolist() == list(pfv.keys())
    assert [ff[fo[i]:fo[i + 1]].tolist() for i in range(len(fn))] == list(pfv.values())
    for f in d[:40]:
        assert ov.transform_one(f, levelsup) == pv.transform1(f, levelsup)


@pytest.mark.parametrize("weighting,scoring", WEIGHTING_SCORING)
def test_oracle_matches_python_restatement_on_real_descriptors(weighting, scoring):
    train, test = _descs()
    arrays = build_vocabulary(train, k=5, L=3, seed=1, stop_frac=0.2)
    ov = OracleVocabulary.create(5, 3, scoring, weighting, *arrays)
    pv = PyVocabulary(5, 3, scoring, weighting, *arrays)
    for levelsup in (0, 1, 2, 3, 5):
        _check_same(ov, pv, test[:150], levelsup)


def test_oracle_matches_python_restatement_with_ties_and_shallow_leaves():
    rng = np.random.default_rng(3)
    arrays = random_vocabulary(4, 3, seed=2, bits=24)  # sparse descriptors: many equal distances
    ov = OracleVocabulary.create(4, 3, 0, 0, *arrays)
    pv = PyVocabulary(4, 3, 0, 0, *arrays)
    feats = np.zeros((120, 32), np.uint8)
    for i in range(120):
        for b in rng.choice(256, size=20, replace=False):
            feats[i, b // 8] |= np.uint8(1 << (b % 8))
    _check_same(ov, pv, feats, 1)
    train = _descs(1, nf=300, stream=31)[0]
    arrays = build_vocabulary(train, k=3, L=4, seed=5, shallow_leaves=True)
    ov = OracleVocabulary.create(3, 4, 0, 0, *arrays)
    pv = PyVocabulary(3, 4, 0, 0, *arrays)
    _check_same(ov, pv, train[:100], 2)  # leaves above nid_level: nid = the leaf


def _kat_vocabulary():
    z, f = np.zeros(32, np.uint8), np.full(32, 255, np.uint8)
    a1 = z.copy()
    a1[0] = 255
    b1 = f.copy()
    b1[0] = 0
    parent = [0, 0, 1, 1, 2, 2]  # 1 = A, 2 = B, 3 = A0, 4 = A1, 5 = B0, 6 = B1
    leaf = [0, 0, 1, 1, 1, 1]  # words: A0 = 0, A1 = 1, B0 = 2, B1 = 3
    desc = np.stack([z, f, z, a1, f, b1])
    weight = [0.0, 0.0, 1.0, 2.0, 0.0, 0.5]  # B0 is a stop word
    return parent, leaf, desc, weight


def test_oracle_known_answer():
    """Hand-computed transform of a 2-level binary vocabulary (TemplatedVocabulary.h:1126-1259)."""
    ov = OracleVocabulary.create(2, 2, 0, 0, *_kat_vocabulary())
    z, f = np.zeros(32, np.uint8), np.full(32, 255, np.uint8)
    f2 = z.copy()
    f2[0] = 255
    f4 = f.copy()
    f4[0] = 0
    tie = z.copy()
    tie[:16] = 255  # distance 128 to A and to B: strict `<` keeps A; then A1 (120) beats A0 (128)
    feats = np.stack([z, f2, f, f4, z, tie])
    assert ov.transform_one(z, 1) == (0, 1.0, 1)
    assert ov.transform_one(f, 1) == (2, 0.0, 2)
    assert ov.transform_one(tie, 0) == (1, 2.0, 4)  # nid level L - 0 = the leaf level
    assert ov.transform_one(tie, 2) == (1, 2.0, 0)  # nid level <= 0: the root
    bw, bv, fn, fo, ff = ov.transform(feats, 1)
    assert bw.tolist() == [0, 1, 3]
    assert bv.tolist() == [2.0 / 6.5, 4.0 / 6.5, 0.5 / 6.5]  # L1 of sums 1 + 1, 2 + 2, 0.5
    assert fn.tolist() == [1, 2] and fo.tolist() == [0, 4, 5] and ff.tolist() == [0, 1, 4, 5, 3]


@pytest.mark.parametrize("fmt", ["%.17g", "%g"])
def test_text_format_round_trip(tmp_path, fmt):
    train, test = _descs(stream=32)
    parent, leaf, desc, weight = build_vocabulary(train, k=6, L=3, seed=4, stop_frac=0.1)
    path = tmp_path / "voc.txt"
    write_text(path, 6, 3, 0, 0, parent, leaf, desc, weight, weight_fmt=fmt)
    ov = OracleVocabulary.load_text(path)
    assert ov.info().tolist() == [6, 3, 0, 0, len(parent) + 1, int(leaf.sum())]
    w = weight if fmt == "%.17g" else np.array([float(fmt % x) for x in weight])
    ref = OracleVocabulary.create(6, 3, 0, 0, parent, leaf, desc, w)
    a, b = ov.transform(test, 4), ref.transform(test, 4)
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()
    bad = tmp_path / "bad.txt"
    bad.write_text("30 6 0 0\n")  # k > 20: the reference's header check fails
    assert OracleVocabulary.load_text(bad) is None


def test_product_vocabulary_validates_before_device_work():
    lib = orb.hip_lib()
    h = ctypes.c_void_p()
    parent = np.array([0, 2], np.int32)  # node 2's parent is itself
    leaf = np.array([0, 1], np.uint8)
    desc = np.zeros((2, 32), np.uint8)
    w = np.ones(2)
    p = [x.ctypes.data_as(ctypes.c_void_p) for x in (parent, leaf, desc, w)]
    assert lib.orb_vocabulary_create(10, 6, 0, 0, 2, *p, 0, ctypes.byref(h)) == _native.ORB_EINVAL
    parent[1] = 1
    assert lib.orb_vocabulary_create(25, 6, 0, 0, 2, *p, 0, ctypes.byref(h)) == _native.ORB_EINVAL  # k > 20
    assert lib.orb_vocabulary_create(10, 0, 0, 0, 2, *p, 0, ctypes.byref(h)) == _native.ORB_EINVAL  # L < 1
    assert lib.orb_vocabulary_load_text(b"/nonexistent/voc.txt", 0, ctypes.byref(h)) == _native.ORB_EINVAL
    v = orb.ORBVocabulary()
    assert v.loadFromTextFile("/nonexistent/voc.txt") is False and v.empty()
