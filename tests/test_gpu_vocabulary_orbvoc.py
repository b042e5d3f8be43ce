"""The DBoW2 vocabulary at ORBvoc.txt's shape: k = 10, L = 6, 1 111 111 nodes, 10^6 words
(TemplatedVocabulary.h:1126-1259, 1338-1424; Data/ORBvoc.txt itself is absent from the
reference).  The tree is random (random_vocabulary: complete, random node
descriptors, random leaf weights) — the descent does the same work per level on any tree of
this shape, and it is ~55 MB on the device, far past one XCD's L2, as ORBvoc is.  Parity
against the oracle (oracle/orb_oracle_voc.cpp) on real extractor descriptors and on random
ones, per feature and per frame (BowVector doubles bit for bit, FeatureVector CSR), single and
batched, and through a 156 MB text file read by both loaders."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.vocabulary import write_text
from oracle_lib import Oracle
from vocab_util import OracleVocabulary, random_vocabulary

pytestmark = pytest.mark.gpu

K, L = 10, 6


@pytest.fixture(scope="module")
def voc():
    arrays = random_vocabulary(K, L, seed=106)
    gv = orb.ORBVocabulary.from_arrays(K, L, 0, 0, *arrays)  # TF_IDF, L1_NORM (ORBvoc.txt's header)
    ov = OracleVocabulary.create(K, L, 0, 0, *arrays)
    assert gv.size() == 10**6 and gv.n_nodes == 1111111
    return arrays, gv, ov


@pytest.fixture(scope="module")
def descs():
    ora = Oracle(1000, 1.2, 8, 1, 20)
    real = [ora.extract(f)[1] for f in orb.synth_stream(640, 480, stream=41, first=0, count=4)]
    rnd = np.random.default_rng(6).integers(0, 256, size=(1000, 32), dtype=np.uint8)
    return real + [rnd]


def _same(gv, ov, d, levelsup):
    bow, fv = gv.transform(d, levelsup)
    bw, bv, fn, fo, ff = ov.transform(d, levelsup)
    assert list(bow.keys()) == bw.tolist()
    assert np.array(list(bow.values()), np.float64).view(np.uint64).tolist() == bv.view(np.uint64).tolist()
    assert fv.nodes.tolist() == fn.tolist() and fv.offsets.tolist() == fo.tolist()
    assert fv.features.tolist() == ff.tolist()


@pytest.mark.parametrize("levelsup", [0, 2, 4, 6])
def test_orbvoc_scale_transform_parity(voc, descs, levelsup):
    _, gv, ov = voc
    for d in descs:
        _same(gv, ov, d, levelsup)


def test_orbvoc_scale_per_feature_parity(voc, descs):
    import torch

    _, gv, ov = voc
    d = descs[0]
    w, wt, nd = gv.transform_features_device(torch.from_numpy(np.ascontiguousarray(d)).cuda(), 4)
    torch.cuda.synchronize()
    w, wt, nd = w.cpu().numpy().view(np.uint32), wt.cpu().numpy(), nd.cpu().numpy().view(np.uint32)
    for i, f in enumerate(d):
        assert (int(w[i]), float(wt[i]), int(nd[i])) == ov.transform_one(f, 4), i


def test_orbvoc_scale_batch_device_parity(voc, descs):
    import torch

    _, gv, ov = voc
    cap, B = 1000, 6
    D = np.zeros((B, cap, 32), np.uint8)
    srcs = [descs[0], descs[1], None, descs[2][:333], descs[3], descs[4]]
    counts = np.array([0 if s is None else len(s) for s in srcs], np.int32)
    for b, s in enumerate(srcs):
        if s is not None:
            D[b, :len(s)] = s
    o = gv.transform_batch_device(torch.from_numpy(D).cuda(), torch.from_numpy(counts).cuda(), 4)
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in o.items()}
    for b in range(B):
        bw, bv, fn, fo, ff = ov.transform(D[b, :counts[b]], 4)
        nb, nf = int(o["bow_n"][b]), int(o["fv_n"][b])
        assert o["bow_words"][b, :nb].view(np.uint32).tolist() == bw.tolist()
        assert o["bow_values"][b, :nb].view(np.uint64).tolist() == bv.view(np.uint64).tolist()
        assert o["fv_nodes"][b, :nf].view(np.uint32).tolist() == fn.tolist()
        assert o["fv_offsets"][b, :nf + 1].tolist() == fo.tolist()
        assert o["fv_features"][b, :fo[-1]].tolist() == ff.tolist()


def test_orbvoc_scale_text_load(voc, descs, tmp_path):
    """loadFromTextFile on an ORBvoc-sized text (the reference's ~6 significant weight digits)."""
    arrays, _, _ = voc
    path = tmp_path / "ORBvoc_synthetic.txt"
    write_text(path, K, L, 0, 0, *arrays, weight_fmt="%g")
    gv = orb.ORBVocabulary()
    assert gv.loadFromTextFile(str(path))
    ov = OracleVocabulary.load_text(path)
    assert (gv.k, gv.L, gv.n_nodes, gv.n_words) == (K, L, 1111111, 10**6)
    _same(gv, ov, descs[1], 4)
