"""GPU parity of the Frame keypoint geometry (csrc/orb_frame.hip) and of the calibrated-camera
front end: extraction -> UndistortKeyPoints -> SearchForInitialization on mvKeysUn with the
ComputeImageBounds grid (Frame.cc:56-128, 289-349; ORBmatcher.cc:598-713), bit-exact against
the oracle.  cv::undistortPoints is parity-unpinned against a real OpenCV 2.4:
the oracle restatement is pinned by tests/test_undistort_oracle.py."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd import camera
from oracle_lib import Oracle, compute_image_bounds, search_for_initialization, undistort_keypoints, undistort_points

pytestmark = pytest.mark.gpu

K_VGA = (458.654, 457.296, 320.215, 238.375)
D_SYN = (-0.2, 0.05, 0.0005, -0.0003)  # synthetic k1 = -0.2, k2 = 0.05 (+ small tangential)
CAMS = [
    (K_VGA, D_SYN),
    ((718.856, 718.856, 607.1928, 185.2157), (-0.3, 0.1, 0.001, -0.0005)),
    ((320.0, 320.0, 320.0, 240.0), (-0.35, 0.12, -0.002, 0.003)),
    ((500.0, 480.0, 300.5, 260.25), (0.15, -0.02, 0.0, 0.0)),
    # strong pincushion: keypoints near the edge midpoints undistort outside the corner bounds
    # (21 of 6 synth frames' keypoints at 640x480, oracle)
    ((500.0, 480.0, 300.5, 260.25), (0.45, 0.05, 0.0005, 0.0)),
]


@pytest.mark.parametrize("cam", range(len(CAMS)))
def test_undistort_points_bit_exact(cam):
    K4, d4 = CAMS[cam]
    rng = np.random.default_rng(cam)
    xy = np.concatenate([rng.uniform(-100, 1400, (100_000, 2)),
                         np.array([[0, 0], [1241, 0], [0, 376], [1241, 376], K4[2:4]])]).astype(np.float32)
    assert camera.undistort_points(xy, K4, d4).tobytes() == undistort_points(xy, K4, d4).tobytes()


@pytest.mark.parametrize("cam", range(len(CAMS)))
def test_image_bounds(cam):
    K4, d4 = CAMS[cam]
    for cols, rows in ((640, 480), (752, 480), (1241, 376), (1280, 720)):
        b = camera.compute_image_bounds(cols, rows, K4, d4)
        assert (b.min_x, b.max_x, b.min_y, b.max_y) == compute_image_bounds(cols, rows, K4, d4)
    b = camera.compute_image_bounds(640, 480, K4, (0.0, 0.3, 0.1, 0.1))  # k1 == 0: the rectangle
    assert (b.min_x, b.max_x, b.min_y, b.max_y) == (0, 640, 0, 480)


def test_bad_camera_rejected():
    with pytest.raises(orb.OrbError):
        camera.undistort_points(np.zeros((4, 2), np.float32), (0.0, 1.0, 0.0, 0.0), D_SYN)


def _batch_pipeline(frames, nf, K4, d4):
    import torch

    B, H, W = frames.shape
    ext = orb.ORBextractor(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    kps, desc, cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    kun = camera.undistort_keypoints_batch_device(kps, cnt, K4, d4)
    bounds = camera.compute_image_bounds(W, H, K4, d4)
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(kun, desc, cnt, f1, f1 + 1, W, H, 100,
                                                                               bounds=bounds)
    torch.cuda.synchronize()
    return (kps.cpu().numpy(), kun.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy(), m12.cpu().numpy(),
            nm.cpu().numpy(), (bounds.min_x, bounds.max_x, bounds.min_y, bounds.max_y))


def _check(frames, nf, K4, d4, kps, kun, desc, cnt, m12, nm, bounds):
    B, H, W = frames.shape
    ora = Oracle(nf, 1.2, 8, 1, 20)
    ref = []
    assert bounds == compute_image_bounds(W, H, K4, d4)
    for b in range(B):
        ko, do = ora.extract(frames[b])
        assert kps[b, : cnt[b]].tobytes() == ko.tobytes(), b
        assert desc[b, : cnt[b]].tobytes() == do.tobytes(), b
        ku = undistort_keypoints(ko, K4, d4)
        assert kun[b, : cnt[b]].tobytes() == ku.tobytes(), b
        ref.append((ku, do))
    for p in range(B - 1):
        (k1, d1), (k2, d2) = ref[p], ref[p + 1]
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, d1, k2, d2, W, H, prev, 0.9, True, 100, bounds=bounds)
        assert nm[p] == no and np.array_equal(m12[p, : cnt[p]], m12o), p
    assert (nm > 0).all()


@pytest.mark.parametrize("W,H,nf,cam", [(640, 480, 1000, 0), (1241, 376, 2000, 1), (752, 480, 1000, 2),
                                        (640, 480, 1000, 3), (640, 480, 1000, 4)])
def test_batch_extract_undistort_match(W, H, nf, cam):
    """cams 3 / 4 are pincushion cameras (k1 > 0); with cam 4 undistorted keypoints land outside
    the corner-derived ComputeImageBounds, so k_match_init's PosInGrid rejection on mvKeysUn
    (Frame.cc:267-277) runs."""
    frames = orb.synth_stream(W, H, stream=31, first=0, count=6)
    K4, d4 = CAMS[cam]
    out = _batch_pipeline(frames, nf, K4, d4)
    _check(frames, nf, K4, d4, *out)
    if cam == 4:
        kun, cnt, (x0, x1, y0, y1) = out[1], out[3], out[6]
        outside = 0
        for b in range(len(frames)):
            k = orb.keypoints_from_bytes(kun[b], cnt[b])
            outside += int(((k["x"] < x0) | (k["x"] >= x1) | (k["y"] < y0) | (k["y"] >= y1)).sum())
        assert outside > 0  # the out-of-grid rejection really ran


@pytest.mark.parametrize("cam", [0, 4])
def test_batch_undistorted_reduced_capacity(cam):
    """>= 256 pairs on undistorted keypoints: k_match_init's reduced-LDS-capacity batch (and its
    in-workgroup large-capacity redo) on mvKeysUn inside the camera's bounds, bit-exact."""
    import torch

    W, H, nf = 640, 480, 1000
    K4, d4 = CAMS[cam]
    frames = orb.synth_stream(W, H, stream=35, first=0, count=8)
    ext = orb.ORBextractor(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=8)
    kps, desc, cnt = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    kun = camera.undistort_keypoints_batch_device(kps, cnt, K4, d4)
    bounds = camera.image_bounds(W, H, K4, d4)
    f1 = torch.tensor([b for _ in range(37) for b in range(7)], dtype=torch.int32, device="cuda")
    assert f1.numel() >= 256
    m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(kun, desc, cnt, f1, f1 + 1, W, H, 100,
                                                                               bounds=bounds)
    torch.cuda.synchronize()
    kun, desc, cnt, m12, nm = kun.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()
    bt = (bounds.min_x, bounds.max_x, bounds.min_y, bounds.max_y)
    assert bt == compute_image_bounds(W, H, K4, d4)
    ora = Oracle(nf, 1.2, 8, 1, 20)
    ref = []
    for b in range(8):
        ko, do = ora.extract(frames[b])
        ku = undistort_keypoints(ko, K4, d4)
        assert kun[b, : cnt[b]].tobytes() == ku.tobytes(), b
        ref.append((ku, do))
    expect = []
    for b in range(7):
        (k1, d1), (k2, d2) = ref[b], ref[b + 1]
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        expect.append(search_for_initialization(k1, d1, k2, d2, W, H, prev, 0.9, True, 100, bounds=bt))
    for p in range(f1.numel()):
        no, m12o = expect[p % 7]
        assert nm[p] == no and np.array_equal(m12[p, : cnt[p % 7]], m12o), p
    assert (nm > 0).all()


def test_pipeline_wrapper_undistorted_pincushion():
    """FrontEndPipeline.run_undistorted (the Python binding of
    orb_pipeline_extract_undistort_and_match) with the pincushion camera = oracle."""
    import torch

    W, H, B, nf = 640, 480, 6, 1000
    K4, d4 = CAMS[4]
    frames = orb.synth_stream(W, H, stream=36, first=0, count=B)
    from orbslam_jpminipc_amd.pipeline import FrontEndPipeline

    pl = FrontEndPipeline(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B, n_streams=3)
    cap = pl.max_keypoints
    d = torch.from_numpy(frames).cuda()
    kps = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    kun = torch.empty_like(kps)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
    m12 = torch.empty((B - 1, cap), dtype=torch.int32, device="cuda")
    nm = torch.empty((B - 1,), dtype=torch.int32, device="cuda")
    pl.run_undistorted(d, K4, d4, kps, kun, desc, cnt, m12, nm)
    torch.cuda.synchronize()
    pl.close()
    b = camera.image_bounds(W, H, K4, d4)
    _check(frames, nf, K4, d4, kps.cpu().numpy(), kun.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy(),
           m12.cpu().numpy(), nm.cpu().numpy(), (b.min_x, b.max_x, b.min_y, b.max_y))


def test_batch_k1_zero_copies():
    import torch

    frames = orb.synth_stream(640, 480, stream=32, first=0, count=3)
    kps, kun, desc, cnt, m12, nm, bounds = _batch_pipeline(frames, 1000, K_VGA, (0.0, 0.05, 0.01, 0.0))
    assert bounds == (0, 640, 0, 480)
    for b in range(3):
        assert kun[b, : cnt[b]].tobytes() == kps[b, : cnt[b]].tobytes()
    # in place (d_kps_un == d_kps) is allowed
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=3)
    k, _, c = ext.extract_batch_device(torch.from_numpy(frames).cuda())
    ref = camera.undistort_keypoints_batch_device(k, c, K_VGA, D_SYN)
    camera.undistort_keypoints_batch_device(k, c, K_VGA, D_SYN, d_kps_un=k)
    torch.cuda.synchronize()
    assert torch.equal(k, ref)


def test_pipeline_extract_undistort_and_match():
    """orb_pipeline_extract_undistort_and_match (4 chunk streams) = the serial kernels = oracle."""
    import ctypes

    import torch
    from orbslam_jpminipc_amd._native import FrameBounds, check, hip_lib, ptr

    W, H, B, nf = 640, 480, 8, 1000
    K4, d4 = CAMS[0]
    frames = orb.synth_stream(W, H, stream=33, first=0, count=B)
    L = hip_lib()
    p = ctypes.c_void_p()
    check(L.orb_pipeline_create(nf, 1.2, 8, orb.FAST_SCORE, 20, 0, B, 4, ctypes.byref(p)))
    try:
        cap = L.orb_pipeline_max_keypoints(p)
        d = torch.from_numpy(frames).cuda()
        kps = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
        kun = torch.empty_like(kps)
        desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
        cnt = torch.empty((B,), dtype=torch.int32, device="cuda")
        m12 = torch.empty((B - 1, cap), dtype=torch.int32, device="cuda")
        nm = torch.empty((B - 1,), dtype=torch.int32, device="cuda")
        k4, dd = np.asarray(K4, np.float32), np.asarray(d4, np.float32)
        b = camera.compute_image_bounds(W, H, K4, d4)
        s = torch.cuda.current_stream()
        check(L.orb_pipeline_extract_undistort_and_match(p, B, ptr(d), W, H, W, W * H, ptr(k4), ptr(dd), ptr(kps),
                                                         ptr(kun), ptr(desc), ptr(cnt), FrameBounds(*[b.min_x, b.max_x,
                                                                                                     b.min_y, b.max_y]),
                                                         0.9, 1, 100, ptr(m12), ptr(nm),
                                                         ctypes.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
    finally:
        L.orb_pipeline_destroy(p)
    _check(frames, nf, K4, d4, kps.cpu().numpy(), kun.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy(),
           m12.cpu().numpy(), nm.cpu().numpy(), (b.min_x, b.max_x, b.min_y, b.max_y))


def test_frame_mirror_host_path():
    """Frame(K, distCoef) + ORBmatcher.SearchForInitialization: the reference's per-frame calls
    (Frame::Frame -> UndistortKeyPoints, Tracking::Initialize) through the host entry points."""
    W, H = 640, 480
    K4, d4 = CAMS[0]
    K = np.array([[K4[0], 0, K4[2]], [0, K4[1], K4[3]], [0, 0, 1]], np.float32)
    frames = orb.synth_stream(W, H, stream=34, first=0, count=2)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    F1, F2 = (orb.Frame.from_image(f, ext, K, np.array(d4, np.float32)) for f in frames)
    ora = Oracle(1000, 1.2, 8, 1, 20)
    ref = [ora.extract(f) for f in frames]
    for F, (ko, _) in zip((F1, F2), ref):
        assert F.mvKeys.tobytes() == ko.tobytes()
        assert F.mvKeysUn.tobytes() == undistort_keypoints(ko, K4, d4).tobytes()
        assert (F.mnMinX, F.mnMaxX, F.mnMinY, F.mnMaxY) == compute_image_bounds(W, H, K4, d4)
    prev = np.ascontiguousarray(np.stack([F1.mvKeysUn["x"], F1.mvKeysUn["y"]], 1).astype(np.float32))
    prev_o = prev.copy()
    m12 = []
    n = orb.ORBmatcher(0.9, True).SearchForInitialization(F1, F2, prev, m12, 100)
    no, m12o = search_for_initialization(F1.mvKeysUn, ref[0][1], F2.mvKeysUn, ref[1][1], W, H, prev_o, 0.9, True, 100,
                                         bounds=(F1.mnMinX, F1.mnMaxX, F1.mnMinY, F1.mnMaxY))
    assert n == no > 0 and list(m12) == list(m12o)
    assert prev.tobytes() == prev_o.tobytes()
