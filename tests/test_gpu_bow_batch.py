"""GPU parity of the batched SearchByBoW (csrc/orb_bow.hip, orb_search_by_bow_batch_device)
against the CPU oracle's per-pair SearchByBoW (oracle/orb_oracle_match.cpp, ORBmatcher.cc:155-284
and 715-850): match arrays and counts identical, pair by pair, bit for bit.

Cases: the synthetic scenes of test_gpu_matcher_family (many pairs in one launch, usable flags,
both nnratios / checkOri), nodes with more than 64 candidates (the strided path) and heavy
contention, empty frames, and the real chain extract -> vocabulary transform -> BoW match on
device-resident 640x480 frames (Frame::ComputeBoW, Tracking.cc:927)."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.views import FeatureVector, View
from oracle_lib import OracleMatcher
import scenes as S
from vocab_util import random_vocabulary

pytestmark = pytest.mark.gpu


def _bow_pair(rng, n_pts=500, extra=300, share=0.8):
    V1, V2, P, i1, i2 = S.two_views_of_points(rng, n_pts, n_extra=extra, kmax=45)
    ids = np.sort(rng.choice(10**6, 80, replace=False))
    a_pt = rng.integers(0, len(ids), n_pts)
    a1 = rng.integers(0, len(ids), V1.n)
    a2 = rng.integers(0, len(ids), V2.n)
    a1[i1] = a_pt
    a2[i2] = np.where(rng.random(n_pts) < share, a_pt, rng.integers(0, len(ids), n_pts))
    keep1 = rng.random(len(ids)) < 0.9
    keep2 = rng.random(len(ids)) < 0.9
    a1 = np.where(keep1[a1], a1, np.flatnonzero(keep1)[0])
    a2 = np.where(keep2[a2], a2, np.flatnonzero(keep2)[0])
    fv1, _, _ = S.feature_vector(rng, V1.n, node_ids=ids, assign=a1)
    fv2, _, _ = S.feature_vector(rng, V2.n, node_ids=ids, assign=a2)
    return V1, V2, fv1, fv2


def _pack(views, fvs, usable=None):
    """Frames as the extractor / vocabulary batch entry points lay them out, on the device."""
    import torch

    B = len(views)
    cap = max(1, max(v.n for v in views))
    kps = np.zeros((B, cap, 28), np.uint8)
    desc = np.zeros((B, cap, 32), np.uint8)
    cnt = np.zeros(B, np.int32)
    nodes = np.zeros((B, cap), np.uint32)
    off = np.zeros((B, cap + 1), np.int32)
    feat = np.zeros((B, cap), np.int32)
    fvn = np.zeros(B, np.int32)
    us = np.zeros((B, cap), np.uint8)
    for b, (v, fv) in enumerate(zip(views, fvs)):
        kps[b, : v.n] = np.frombuffer(np.ascontiguousarray(v.kps).tobytes(), np.uint8).reshape(v.n, 28)
        desc[b, : v.n] = v.desc
        cnt[b] = v.n
        nn = len(fv.nodes)
        nodes[b, :nn] = fv.nodes
        off[b, : nn + 1] = fv.offsets
        feat[b, : len(fv.features)] = fv.features
        fvn[b] = nn
        us[b, : v.n] = 1 if usable is None or usable[b] is None else usable[b]
    t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    fv = {"fv_nodes": t(nodes.view(np.int32)), "fv_offsets": t(off), "fv_features": t(feat), "fv_n": t(fvn)}
    return t(kps), t(desc), t(cnt), fv, t(us)


def _run(kf_kf, nn, co, views, fvs, usable, pairs):
    import torch

    d_kps, d_desc, d_cnt, fv, d_us = _pack(views, fvs, usable)
    pa = torch.tensor([a for a, _ in pairs], dtype=torch.int32, device="cuda")
    pb = torch.tensor([b for _, b in pairs], dtype=torch.int32, device="cuda")
    m, n = orb.ORBmatcher(nn, co).search_by_bow_batch_device(kf_kf, d_kps, d_desc, d_cnt, fv, pa, pb,
                                                             d_usable=d_us if usable is not None else None)
    torch.cuda.synchronize()
    m, n = m.cpu().numpy(), n.cpu().numpy()
    o = OracleMatcher(nn, co)
    total = 0
    for p, (a, b) in enumerate(pairs):
        ua = None if usable is None else usable[a]
        ub = None if usable is None else usable[b]
        if kf_kf:
            no, mo = o.SearchByBoW_KF_KF(views[a], ua, fvs[a], views[b], ub, fvs[b])
            rows = views[a].n
        else:
            no, mo = o.SearchByBoW_KF_F(views[a], ua, fvs[a], views[b], fvs[b])
            rows = views[b].n
        assert n[p] == no, (p, n[p], no)
        np.testing.assert_array_equal(m[p, :rows], mo)
        assert (m[p, rows:] == -1).all()
        total += no
    return total


@pytest.mark.parametrize("kf_kf", [False, True])
def test_batch_scenes(kf_kf):
    rng = np.random.default_rng(2100 + kf_kf)
    views, fvs, usable, pairs = [], [], [], []
    for i in range(6):
        V1, V2, fv1, fv2 = _bow_pair(rng)
        views += [V1, V2]
        fvs += [fv1, fv2]
        usable += [(rng.random(V1.n) < 0.8).astype(np.uint8), (rng.random(V2.n) < 0.8).astype(np.uint8)]
        pairs.append((2 * i, 2 * i + 1))
    pairs += [(1, 0), (3, 2), (0, 3)]  # reversed and cross pairs share frames with others
    for nn, co in ((0.75, True), (0.9, False), (0.6, True)):
        assert _run(kf_kf, nn, co, views, fvs, usable, pairs) > 0
        assert _run(kf_kf, nn, co, views, fvs, None, pairs) > 0


@pytest.mark.parametrize("kf_kf", [False, True])
def test_large_nodes_and_contention(kf_kf):
    """One node with 400 queries over 60 candidates (every lane holds a candidate, heavy
    contention for targets) and the reverse, 60 queries over 400 candidates (> 64: the strided
    path with the taken flags in LDS), plus a 200 x 200 node mixed with small ones."""
    rng = np.random.default_rng(7)
    k = S.keypoints(rng, 60, clusters=1, spread=6)
    k["octave"] = 0
    F2 = View(k, S.descriptors(rng, 60), (0, S.W, 0, S.H))
    idx = rng.integers(0, 60, 400)
    F1 = View(F2.kps[idx].copy(), S.perturb(rng, F2.desc[idx], 30), (0, S.W, 0, S.H))
    fv400 = FeatureVector.from_dict({5: list(range(400))})
    fv60 = FeatureVector.from_dict({5: list(range(60))})
    V3 = S.view(rng, 300)
    V4 = View(V3.kps.copy(), S.perturb(rng, V3.desc, 25), (0, S.W, 0, S.H))
    fv3 = FeatureVector.from_dict({1: list(range(0, 200)), 9: list(range(200, 250)), 11: list(range(250, 300))})
    fv4 = FeatureVector.from_dict({1: list(range(100, 300)), 9: list(range(0, 50)), 12: list(range(50, 100))})
    views, fvs = [F1, F2, V3, V4], [fv400, fv60, fv3, fv4]
    pairs = [(0, 1), (1, 0), (2, 3), (3, 2)]
    for nn, co in ((0.99, False), (0.75, True)):
        _run(kf_kf, nn, co, views, fvs, None, pairs)
    assert _run(kf_kf, 0.99, False, views, fvs, None, pairs) > 8


def test_empty_frames():
    rng = np.random.default_rng(3)
    F = S.view(rng, 300)
    E = View(np.zeros(0, orb.KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8), (0, S.W, 0, S.H))
    fvF, _, _ = S.feature_vector(rng, F.n)
    fvE = FeatureVector.from_dict({})
    for kf_kf in (False, True):
        assert _run(kf_kf, 0.7, True, [F, E, F], [fvF, fvE, fvF], None, [(0, 1), (1, 0), (1, 1), (0, 2)]) >= 0


def test_extract_transform_match_chain():
    """640x480 frames on the device -> ORBVocabulary.transform_batch_device (levelsup 4) ->
    batched SearchByBoW(KF = frame t, F = frame t+1) with Tracking.cc:927's nnratio 0.7, every
    pair checked against the oracle run on the same keypoints, descriptors and FeatureVectors."""
    import torch

    B, W, H = 6, 640, 480
    frames = orb.synth_stream(W, H, stream=2, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d_kps, d_desc, d_cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    voc = orb.ORBVocabulary.from_arrays(10, 4, 0, 0, *random_vocabulary(10, 4, seed=11))
    fv = voc.transform_batch_device(d_desc, d_cnt, 2)  # nodes at level L - 2 = 2 (100 nodes, as ORBvoc at levelsup 4)
    pa = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    for kf_kf, nn in ((False, 0.7), (True, 0.75)):
        m, n = orb.ORBmatcher(nn, True).search_by_bow_batch_device(kf_kf, d_kps, d_desc, d_cnt, fv, pa, pa + 1)
        torch.cuda.synchronize()
        m, n = m.cpu().numpy(), n.cpu().numpy()
        kps_h, desc_h, cnt = d_kps.cpu().numpy(), d_desc.cpu().numpy(), d_cnt.cpu().numpy()
        nodes, off, feat, fvn = (fv[k].cpu().numpy() for k in ("fv_nodes", "fv_offsets", "fv_features", "fv_n"))
        views, fvs = [], []
        for b in range(B):
            k = orb.keypoints_from_bytes(kps_h[b], cnt[b])
            views.append(View(k, desc_h[b, : cnt[b]], (0, W, 0, H)))
            fvs.append(FeatureVector(nodes[b, : fvn[b]].view(np.uint32), off[b, : fvn[b] + 1],
                                     feat[b, : off[b, fvn[b]]]))
        o = OracleMatcher(nn, True)
        for p in range(B - 1):
            if kf_kf:
                no, mo = o.SearchByBoW_KF_KF(views[p], None, fvs[p], views[p + 1], None, fvs[p + 1])
                rows = cnt[p]
            else:
                no, mo = o.SearchByBoW_KF_F(views[p], None, fvs[p], views[p + 1], fvs[p + 1])
                rows = cnt[p + 1]
            assert n[p] == no and no > 50, (p, n[p], no)
            np.testing.assert_array_equal(m[p, :rows], mo)
