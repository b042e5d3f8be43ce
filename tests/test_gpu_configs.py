"""GPU parity at the benchmark's own scale and under concurrency.

* the bench's timed workload itself (640x480, B = 512 frames of stream 0, 511 consecutive
  pairs): every frame's keypoints / descriptors and every pair's matches against the oracle;
* SearchForInitialization past k_match_init's LDS capacity (the reference init extractor at
  1280x720: nFeatures*2 = 5000, Tracking.cc:126/217) through the batched device entry point;
* stream ordering of one extractor handle used from two streams, the phase-2
  guard, and matcher calls from several host threads at once (Tracking / LocalMapping /
  LoopClosing run matchers concurrently, main.cc:164-193).
"""
import threading

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle, OracleMatcher, search_for_initialization

pytestmark = pytest.mark.gpu


def _oracle_threads():
    import os

    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box's CPU share is 16


def _oracle_extract_all(frames, nf, threads=None):
    """Oracle extraction of every frame, `threads` oracle instances in parallel (ctypes
    releases the GIL)."""
    out = [None] * len(frames)
    threads = threads or _oracle_threads()

    def work(t):
        ora = Oracle(nf, 1.2, 8, 1, 20)
        for b in range(t, len(frames), threads):
            out[b] = ora.extract(frames[b])

    ts = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def _device_extract_and_match(frames, nf, pairs=None):
    """bench.py's step on `frames`: orb_extract_batch_device, then the batched
    SearchForInitialization over `pairs` (default: every consecutive pair)."""
    import torch

    B, H, W = frames.shape
    ext = orb.ORBextractor(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    kps, desc, cnt = ext.extract_batch_device(d)
    if pairs is None:
        pairs = [(b, b + 1) for b in range(B - 1)]
    f1 = torch.tensor([a for a, _ in pairs], dtype=torch.int32, device="cuda")
    f2 = torch.tensor([b for _, b in pairs], dtype=torch.int32, device="cuda")
    m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(kps, desc, cnt, f1, f2, W, H, 100)
    torch.cuda.synchronize()
    return kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()


def _check_batch(frames, nf, kps, desc, cnt, m12, nm, pairs=None):
    B, H, W = frames.shape
    ref = _oracle_extract_all(frames, nf)
    for b in range(B):
        ko, do = ref[b]
        assert cnt[b] == len(ko), b
        assert kps[b, : cnt[b]].tobytes() == ko.tobytes(), f"frame {b} keypoints"
        assert desc[b, : cnt[b]].tobytes() == do.tobytes(), f"frame {b} descriptors"
    if pairs is None:
        pairs = [(b, b + 1) for b in range(B - 1)]
    for p, (a, b) in enumerate(pairs):
        k1, d1 = ref[a]
        k2, d2 = ref[b]
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, d1, k2, d2, W, H, prev, 0.9, True, 100)
        assert nm[p] == no, p
        assert np.array_equal(m12[p, : cnt[a]], m12o), p


def _bench_stream_batch(W, H, streams, per):
    """bench.py's frames and pairs for `streams` camera streams of `per` frames each (c5 at
    N ranks: rank r owns streams r, r + N, ...; c3 / c4: one stream = the rank)."""
    frames = np.concatenate([orb.synth_stream(W, H, stream=s, first=0, count=per) for s in streams])
    pairs = [(k * per + t, k * per + t + 1) for k in range(len(streams)) for t in range(per - 1)]
    return frames, pairs


def test_bench_batch_full_parity():
    """bench.py's default timed batch, as bench.py builds it (synth_stream(640, 480, stream=rank
    0, first 0, count 512)): all 512 frames and all 511 pairs bit-exact."""
    frames = orb.synth_stream(640, 480, stream=0, first=0, count=512)
    _check_batch(frames, 1000, *_device_extract_and_match(frames, 1000))


def test_bench_batch_c4_full_parity():
    """bench.py --workload c4's timed batch: 512 KITTI-shaped 1241x376 frames of stream 0,
    ORBextractor(2000, 1.2, 8), 511 consecutive pairs.  Exercises k_rerun at its large-batch
    workgroup count and k_match_init's reduced LDS capacity (P >= 256) at this geometry: every
    frame and every pair bit-exact."""
    frames, pairs = _bench_stream_batch(1241, 376, [0], 512)
    _check_batch(frames, 2000, *_device_extract_and_match(frames, 2000, pairs), pairs=pairs)


def _check_sampled(frames, nf, per, kps, desc, cnt, m12, nm, pairs, every=16):
    """_check_batch on a sample of a stream batch: within each stream of `per` frames the pairs
    (t, t+1) with t % every == 0 plus the stream's last pair, and every frame those pairs touch
    (so each stream's first and last frame are always in).  The device ran the whole batch;
    only the oracle side is sampled."""
    B, H, W = frames.shape
    sel_pairs = [p for p, (a, _) in enumerate(pairs) if (a % per) % every == 0 or (a % per) == per - 2]
    sel_frames = sorted({f for p in sel_pairs for f in pairs[p]})
    pos = {f: i for i, f in enumerate(sel_frames)}
    ref = _oracle_extract_all(frames[sel_frames], nf)
    for f in sel_frames:
        ko, do = ref[pos[f]]
        assert cnt[f] == len(ko), f
        assert kps[f, : cnt[f]].tobytes() == ko.tobytes(), f"frame {f} keypoints"
        assert desc[f, : cnt[f]].tobytes() == do.tobytes(), f"frame {f} descriptors"
    for p in sel_pairs:
        a, b = pairs[p]
        k1, d1 = ref[pos[a]]
        k2, d2 = ref[pos[b]]
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, d1, k2, d2, W, H, prev, 0.9, True, 100)
        assert nm[p] == no, p
        assert np.array_equal(m12[p, : cnt[a]], m12o), p
    return len(sel_frames), len(sel_pairs)


def test_bench_batch_c5_full_parity():
    """8 independent 1280x720 streams x 128 frames (B = 1024), ORBextractor(2500, 1.2, 8), the
    8 x 127 within-stream pairs: every frame and every pair bit-exact (a smaller batch than
    bench.py's default c5 step; that one is test_bench_batch_c5_default_step_sampled)."""
    frames, pairs = _bench_stream_batch(1280, 720, range(8), 128)
    _check_batch(frames, 2500, *_device_extract_and_match(frames, 2500, pairs), pairs=pairs)


def test_bench_batch_c5_default_step_sampled():
    """bench.py --workload c5's default timed step at N = 1, exactly as bench.py builds it: the
    8 streams x 512 frames (--frames-per-stream 512, B = 4096: k_pyr_stream, k_rerun's
    large-batch workgroup count and k_match_init's reduced LDS capacity over 8 x 511 pairs).
    The device runs the whole step; the oracle checks every 16th within-stream pair plus each
    stream's last pair, and every frame those pairs touch, bit-exact."""
    per = 512
    frames, pairs = _bench_stream_batch(1280, 720, range(8), per)
    out = _device_extract_and_match(frames, 2500, pairs)
    nfr, npr = _check_sampled(frames, 2500, per, *out, pairs=pairs)
    assert nfr >= 8 * 34 and npr >= 8 * 33, (nfr, npr)


@pytest.mark.parametrize("rank", [3])
def test_bench_batch_c5_rank_of_eight_parity(rank):
    """c5 at N = 8 as bench.py runs it: one rank's load is one stream of 512 frames (B = 512,
    511 pairs; replicas.streams_of_rank(8, rank, 8) = [rank]) at 1280x720, which takes
    k_pyr_stream (B >= 256) and the reduced-capacity matcher (P >= 256) at this geometry.  Every
    frame and every pair bit-exact."""
    from orbslam_jpminipc_amd import replicas

    streams = replicas.streams_of_rank(8, rank, 8)
    assert list(streams) == [rank]
    frames, pairs = _bench_stream_batch(1280, 720, streams, 512)
    _check_batch(frames, 2500, *_device_extract_and_match(frames, 2500, pairs), pairs=pairs)


def test_match_batch_device_over_lds_capacity():
    """1280x720 with the init extractor's 5000 features: > 1024 octave-0 keypoints per frame,
    so every pair goes through k_match_init_big."""
    frames = orb.synth_stream(1280, 720, stream=6, first=0, count=4)
    kps, desc, cnt, m12, nm = _device_extract_and_match(frames, 5000)
    oct0 = [int((orb.keypoints_from_bytes(kps[b], cnt[b])["octave"] == 0).sum()) for b in range(len(frames))]
    assert max(oct0) > 1024, oct0  # the fallback really ran
    assert (nm > 0).all()
    _check_batch(frames, 5000, kps, desc, cnt, m12, nm)


def test_extractor_two_streams_no_sync():
    """A device launch on a side stream immediately followed by host-buffer extractions on the
    same handle (no synchronisation in between): the handle orders its workspace users."""
    import torch

    B = 4
    frames = orb.synth_stream(640, 480, stream=12, first=0, count=B)
    other = orb.synth_stream(640, 480, stream=13, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    ref = ext.extract_batch(frames)
    side = torch.cuda.Stream()
    d_other = torch.from_numpy(other).cuda()
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(side):
            ko, do, co = ext.extract_batch_device(d_other, stream=side)
        got = ext.extract_batch(frames)  # host entry point, handle stream, no sync before it
        for b in range(B):
            assert got[b][0].tobytes() == ref[b][0].tobytes()
            assert got[b][1].tobytes() == ref[b][1].tobytes()
        side.synchronize()
    # and the device result on the side stream is itself intact
    ora = Oracle(1000, 1.2, 8, 1, 20)
    c = co.cpu().numpy()
    for b in range(B):
        k, d = ora.extract(other[b])
        assert ko[b, : c[b]].cpu().numpy().tobytes() == k.tobytes()


def test_phase2_without_pyramid_rejected():
    import torch

    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=4)
    d = torch.from_numpy(orb.synth_stream(640, 480, stream=1, count=4)).cuda()
    ext.set_phases(2)
    with pytest.raises(Exception):
        ext.extract_batch_device(d)
    ext.set_phases(1)
    ext.extract_batch_device(d[:2])
    ext.set_phases(2)
    with pytest.raises(Exception):  # pyramid of 2 frames only
        ext.extract_batch_device(d)
    ext.extract_batch_device(d[:2])
    ext.set_phases(3)
    torch.cuda.synchronize()


def test_matchers_from_three_threads():
    """WindowSearch (Tracking), SearchForTriangulation (LocalMapping) and SearchByBoW KF-KF
    (LoopClosing) run concurrently from three host threads, plus a fourth running
    SearchForInitialization; each repeated, each bit-exact against the oracle."""
    import scenes as S
    from test_gpu_matcher_family import _bow_pair
    from orbslam_jpminipc_amd.views import View

    rng = np.random.default_rng(77)
    F2 = S.view(rng, 1000, clusters=6, spread=20)
    idx = rng.integers(0, F2.n, 900)
    k1 = F2.kps[idx].copy()
    k1["x"] = np.clip(k1["x"] + rng.normal(0, 4, len(idx)), 0, S.W - 1)
    k1["y"] = np.clip(k1["y"] + rng.normal(0, 4, len(idx)), 0, S.H - 1)
    F1 = View(k1, S.perturb(rng, F2.desc[idx], 80), (0, S.W, 0, S.H))
    V1, V2, fv1, fv2 = _bow_pair(rng, n_pts=600, extra=200, share=0.9)
    F12 = S.fundamental12(V1, V2)
    h1 = (rng.random(V1.n) < 0.3).astype(np.uint8)
    h2 = (rng.random(V2.n) < 0.3).astype(np.uint8)
    u1 = (rng.random(V1.n) < 0.8).astype(np.uint8)
    u2 = (rng.random(V2.n) < 0.8).astype(np.uint8)
    frames = orb.synth_stream(640, 480, stream=8, count=2)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    Fa, Fb = (orb.Frame.from_image(f, ext) for f in frames)
    prev0 = np.ascontiguousarray(np.stack([Fa.mvKeys["x"], Fa.mvKeys["y"]], 1).astype(np.float32))

    jobs = {
        "window": (lambda M: M.WindowSearch(F1, None, F2, 100), 0.9),
        "triang": (lambda M: M.SearchForTriangulation(V1, h1, fv1, V2, h2, fv2, F12), 0.6),
        "bow": (lambda M: M.SearchByBoW_KF_KF(V1, u1, fv1, V2, u2, fv2), 0.75),
    }
    expect = {k: f(OracleMatcher(nn, True)) for k, (f, nn) in jobs.items()}
    p = prev0.copy()
    expect["sfi"] = search_for_initialization(Fa.mvKeys, Fa.mDescriptors, Fb.mvKeys, Fb.mDescriptors, 640, 480, p,
                                              0.9, True, 100)
    errors = []
    start = threading.Barrier(4)

    def run(name):
        try:
            start.wait()
            for _ in range(10):
                if name == "sfi":
                    p = prev0.copy()
                    m12 = []
                    n = orb.ORBmatcher(0.9, True).SearchForInitialization(Fa, Fb, p, m12, 100)
                    got = (n, np.array(m12, np.int32))
                else:
                    f, nn = jobs[name]
                    got = f(orb.ORBmatcher(nn, True))
                ne, oe = expect[name]
                assert got[0] == ne and np.array_equal(got[1], oe), name
        except Exception as e:  # reported by the main thread
            errors.append((name, repr(e)))

    ts = [threading.Thread(target=run, args=(n,)) for n in ("window", "triang", "bow", "sfi")]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_match_batch_reduced_capacity_fallback():
    """Batches of >= 256 pairs size k_match_init's LDS for 0.225 x the keypoint capacity of
    octave-0 keypoints.  scaleFactor 1.5 over 5 levels keeps 0.38 x nFeatures at level 0, so
    every pair of a 301-pair batch overflows it and is redone by k_match_init_big: bit-exact."""
    import torch

    frames = orb.synth_stream(640, 480, stream=21, first=0, count=8)
    ext = orb.ORBextractor(1000, 1.5, 5, orb.FAST_SCORE, 20, device=0, max_batch=8)
    d_kps, d_desc, d_cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    f1 = torch.tensor([b for _ in range(43) for b in range(7)], dtype=torch.int32, device="cuda")
    m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(d_kps, d_desc, d_cnt, f1, f1 + 1,
                                                                               640, 480, 100)
    torch.cuda.synchronize()
    kps, desc, cnt = d_kps.cpu().numpy(), d_desc.cpu().numpy(), d_cnt.cpu().numpy()
    m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
    ora = Oracle(1000, 1.5, 5, 1, 20)
    ref = [ora.extract(f) for f in frames]
    oct0 = [int((r[0]["octave"] == 0).sum()) for r in ref]
    assert min(oct0) > 0.225 * ext.max_keypoints and min(oct0) > 256, oct0  # the fallback really runs
    for b in range(8):
        assert kps[b, : cnt[b]].tobytes() == ref[b][0].tobytes()
    for p in range(len(f1)):
        b = p % 7
        k1, d1 = ref[b]
        k2, d2 = ref[b + 1]
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, d1, k2, d2, 640, 480, prev, 0.9, True, 100)
        assert nm[p] == no and np.array_equal(m12[p, : cnt[b]], m12o), p
