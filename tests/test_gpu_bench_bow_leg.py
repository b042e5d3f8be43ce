"""Parity of bench.py's BoW leg at the size it is timed (BENCH `bow`): the c3 step's 512
frames of synthetic stream 0 (640x480, 1000 kp), the ORBvoc-shaped vocabulary of
`bench.orbvoc_shaped_tree` (k = 10, L = 6, 1 111 111 nodes, TF-IDF / L1), the batched
transform at levelsup 4 (Frame::ComputeBoW, Frame.cc:280-287; TemplatedVocabulary.h:1126-1259),
then the batched SearchByBoW(KF = frame t, F = frame t+1) of all 511 pairs with
TrackReferenceKeyFrame's ORBmatcher(0.7, true) (Tracking.cc:927; ORBmatcher.cc:155-284), run
exactly as `bench.bow_leg` runs it.  Checked against the oracle: the FeatureVectors of the
sampled frames (oracle transform on the same descriptors), and the match rows and counts of 40
sampled pairs plus the first and the last pair (the oracle's SearchByBoW on the device's
keypoints, descriptors and FeatureVectors); the extraction of the sampled frames against the
oracle's extractor as well."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.views import FeatureVector, View
from oracle_lib import Oracle, OracleMatcher
from vocab_util import OracleVocabulary

pytestmark = pytest.mark.gpu

W, H, NF, B = 640, 480, 1000, 512


def test_bench_bow_leg_parity():
    import torch

    import bench

    frames = orb.synth_stream(W, H, stream=0, first=0, count=B)  # bench.run_rank, rank 0, c3
    ext = orb.ORBextractor(NF, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d_kps, d_desc, d_cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    arrays = bench.orbvoc_shaped_tree()
    voc = orb.ORBVocabulary.from_arrays(10, 6, 0, 0, *arrays)
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    f2 = f1 + 1
    fv = voc.transform_batch_device(d_desc, d_cnt, 4)
    m, n = orb.ORBmatcher(0.7, True).search_by_bow_batch_device(False, d_kps, d_desc, d_cnt, fv, f1, f2)
    torch.cuda.synchronize()
    m, n = m.cpu().numpy(), n.cpu().numpy()
    kps_h, desc_h, cnt = d_kps.cpu().numpy(), d_desc.cpu().numpy(), d_cnt.cpu().numpy()
    nodes, off, feat, fvn = (fv[k].cpu().numpy() for k in ("fv_nodes", "fv_offsets", "fv_features", "fv_n"))

    rng = np.random.default_rng(2026)
    pairs = sorted(set([0, B - 2] + rng.choice(B - 1, 40, replace=False).tolist()))
    need = sorted(set(pairs) | set(p + 1 for p in pairs))
    ov = OracleVocabulary.create(10, 6, 0, 0, *arrays)
    ora = Oracle(NF, 1.2, 8, 1, 20)
    views, fvs = {}, {}
    for b in need[:8]:  # the extraction itself, on a few of the sampled frames
        ko, do = ora.extract(frames[b])
        assert cnt[b] == len(ko)
        assert kps_h[b, : cnt[b]].tobytes() == ko.tobytes() and desc_h[b, : cnt[b]].tobytes() == do.tobytes(), b
    for b in need:
        k = orb.keypoints_from_bytes(kps_h[b], cnt[b])
        d = desc_h[b, : cnt[b]]
        views[b] = View(k, d, (0, W, 0, H))
        fvs[b] = FeatureVector(nodes[b, : fvn[b]].view(np.uint32), off[b, : fvn[b] + 1], feat[b, : off[b, fvn[b]]])
        _, _, fn, fo, ff = ov.transform(np.ascontiguousarray(d), 4)
        assert fvs[b].nodes.tolist() == fn.tolist() and fvs[b].offsets.tolist() == fo.tolist(), b
        assert fvs[b].features.tolist() == ff.tolist(), b
    o = OracleMatcher(0.7, True)
    total = 0
    for p in pairs:
        no, mo = o.SearchByBoW_KF_F(views[p], None, fvs[p], views[p + 1], fvs[p + 1])
        assert n[p] == no, (p, n[p], no)
        np.testing.assert_array_equal(m[p, : cnt[p + 1]], mo)
        total += no
    assert total > 50 * len(pairs)  # real matching work in every checked pair on average
