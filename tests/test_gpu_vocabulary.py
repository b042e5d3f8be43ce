"""GPU parity of the DBoW2 vocabulary path (csrc/orb_voc.hip) against the CPU oracle
(oracle/orb_oracle_voc.cpp): per-feature word / weight / node, BowVector values as double
bit patterns, FeatureVector CSR, on vocabularies built from real ORB descriptors and on
tie-heavy random trees, for every weighting and the normalising / non-normalising scorings."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.vocabulary import write_text
from oracle_lib import Oracle
from vocab_util import OracleVocabulary, build_vocabulary, random_vocabulary

pytestmark = pytest.mark.gpu

_CACHE = {}


def _frames_desc(n=6, W=640, H=480, nf=1000, stream=40):
    key = (n, W, H, nf, stream)
    if key not in _CACHE:
        ora = Oracle(nf, 1.2, 8, 1, 20)
        _CACHE[key] = [ora.extract(f)[1] for f in orb.synth_stream(W, H, stream=stream, first=0, count=n)]
    return _CACHE[key]


def _vocab(k, L, scoring, weighting, arrays):
    return (orb.ORBVocabulary.from_arrays(k, L, scoring, weighting, *arrays),
            OracleVocabulary.create(k, L, scoring, weighting, *arrays))


def _same_transform(gv, ov, d, levelsup):
    bow, fv = gv.transform(d, levelsup)
    bw, bv, fn, fo, ff = ov.transform(d, levelsup)
    assert list(bow.keys()) == bw.tolist()
    assert np.array(list(bow.values()), np.float64).view(np.uint64).tolist() == bv.view(np.uint64).tolist()
    assert fv.nodes.tolist() == fn.tolist() and fv.offsets.tolist() == fo.tolist()
    assert fv.features.tolist() == ff.tolist()


def _same_features(gv, ov, d, levelsup):
    import torch

    dd = torch.from_numpy(np.ascontiguousarray(d)).cuda()
    w, wt, nd = gv.transform_features_device(dd, levelsup)
    torch.cuda.synchronize()
    w, wt, nd = w.cpu().numpy().view(np.uint32), wt.cpu().numpy(), nd.cpu().numpy().view(np.uint32)
    for i, f in enumerate(d):
        ow, owt, ond = ov.transform_one(f, levelsup)
        assert (int(w[i]), float(wt[i]), int(nd[i])) == (ow, owt, ond), i


@pytest.mark.parametrize("weighting,scoring", [(0, 0), (1, 0), (2, 0), (3, 0), (0, 1), (1, 5), (3, 5), (0, 3)])
def test_vocabulary_transform_parity(weighting, scoring):
    descs = _frames_desc()
    arrays = build_vocabulary(np.concatenate(descs[:3]), k=10, L=4, seed=7, stop_frac=0.1)
    gv, ov = _vocab(10, 4, scoring, weighting, arrays)
    assert gv.size() == int(arrays[1].sum()) and gv.height == 4
    for levelsup in (0, 2, 4, 6):
        for d in descs[3:]:
            _same_transform(gv, ov, d, levelsup)
    _same_features(gv, ov, descs[4], 4)


@pytest.mark.parametrize("k,L,bits", [(16, 3, 256), (20, 2, 256), (9, 4, 24), (20, 3, 16)])
def test_vocabulary_wide_and_tie_heavy_trees(k, L, bits):
    """k > 16 children (lanes loop), sparse random descriptors (many equal distances)."""
    arrays = random_vocabulary(k, L, seed=k + L, bits=bits)
    gv, ov = _vocab(k, L, 0, 0, arrays)
    rng = np.random.default_rng(k)
    if bits >= 256:
        feats = rng.integers(0, 256, size=(700, 32), dtype=np.uint8)
    else:
        feats = np.zeros((700, 32), np.uint8)
        for i in range(700):
            for b in rng.choice(256, size=bits, replace=False):
                feats[i, b // 8] |= np.uint8(1 << (b % 8))
    _same_features(gv, ov, feats, 1)
    _same_transform(gv, ov, feats, 1)


def test_vocabulary_shallow_leaves_and_stop_words():
    descs = _frames_desc()
    arrays = build_vocabulary(descs[0], k=4, L=5, seed=9, shallow_leaves=True, stop_frac=0.4)
    gv, ov = _vocab(4, 5, 0, 0, arrays)
    _same_features(gv, ov, descs[1], 2)
    _same_transform(gv, ov, descs[1], 2)


def test_vocabulary_batch_device_parity():
    import torch

    descs = _frames_desc()
    arrays = build_vocabulary(np.concatenate(descs[:2]), k=10, L=4, seed=11, stop_frac=0.05)
    gv, ov = _vocab(10, 4, 0, 0, arrays)
    cap = 1000
    B = 5
    D = np.zeros((B, cap, 32), np.uint8)
    counts = np.array([len(descs[2]), 0, len(descs[3]), 17, len(descs[5])], np.int32)
    for b, src in enumerate([descs[2], None, descs[3], descs[4][:17], descs[5]]):
        if src is not None:
            D[b, :len(src)] = src
    out = gv.transform_batch_device(torch.from_numpy(D).cuda(), torch.from_numpy(counts).cuda(), 4)
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    for b in range(B):
        bw, bv, fn, fo, ff = ov.transform(D[b, :counts[b]], 4)
        nb, nf = int(o["bow_n"][b]), int(o["fv_n"][b])
        assert o["bow_words"][b, :nb].view(np.uint32).tolist() == bw.tolist()
        assert o["bow_values"][b, :nb].view(np.uint64).tolist() == bv.view(np.uint64).tolist()
        assert o["fv_nodes"][b, :nf].view(np.uint32).tolist() == fn.tolist()
        assert o["fv_offsets"][b, :nf + 1].tolist() == fo.tolist()
        assert o["fv_features"][b, :fo[-1]].tolist() == ff.tolist()


def test_vocabulary_text_load_on_gpu(tmp_path):
    descs = _frames_desc()
    parent, leaf, desc, weight = build_vocabulary(descs[0], k=8, L=3, seed=13)
    path = tmp_path / "voc.txt"
    write_text(path, 8, 3, 0, 0, parent, leaf, desc, weight, weight_fmt="%g")
    gv = orb.ORBVocabulary()
    assert gv.loadFromTextFile(str(path))
    ov = OracleVocabulary.load_text(path)
    assert (gv.k, gv.L, gv.n_nodes, gv.n_words) == (8, 3, len(parent) + 1, int(leaf.sum()))
    _same_transform(gv, ov, descs[2], 4)
    (tmp_path / "blank.txt").write_text(path.read_text() + "\n\n")  # trailing blank lines are skipped
    gv2 = orb.ORBVocabulary()
    assert gv2.loadFromTextFile(str(tmp_path / "blank.txt")) and gv2.n_nodes == gv.n_nodes


def test_empty_vocabulary():
    v = orb.ORBVocabulary.from_arrays(10, 2, 0, 0, [0], [0], np.zeros((1, 32), np.uint8), [0.0])
    assert v.empty()
    bow, fv = v.transform(np.zeros((3, 32), np.uint8))
    assert bow == {} and len(fv.nodes) == 0
