"""GPU parity: the HIP path through the C ABI vs the CPU oracle, bit-exact.

Keypoints are compared as raw 28-byte records (all 7 cv::KeyPoint fields, float bit
patterns), descriptors byte-by-byte, matches index-by-index.
"""
import ctypes

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle, search_for_initialization

pytestmark = pytest.mark.gpu


def _diagnose(ext, ora, img, kg, ko):
    """Localise the first differing stage: pyramid level, then per-cell FAST counts."""
    lib = orb.hip_lib()
    lines = []
    for l in range(ext.nlevels):
        w, h = ctypes.c_int(), ctypes.c_int()
        lib.orb_debug_level_image(ext._h, 0, l, None, ctypes.byref(w), ctypes.byref(h))
        g = np.empty((h.value + 32, w.value + 32), np.uint8)
        lib.orb_debug_level_image(ext._h, 0, l, g.ctypes.data_as(ctypes.c_void_p), ctypes.byref(w), ctypes.byref(h))
        o = ora.level_image(l)
        if g.shape != o.shape or not np.array_equal(g, o):
            bad = np.argwhere(g != o) if g.shape == o.shape else "shape"
            lines.append(f"level {l} image differs: {bad[:5] if not isinstance(bad, str) else bad}")
            break
        cnt = np.zeros(4096, np.int32)
        n = lib.orb_debug_cell_counts(ext._h, 0, l, cnt.ctypes.data_as(ctypes.c_void_p), 4096)
        oc = ora.cell_counts(l).reshape(-1)
        if n != oc.size or not np.array_equal(cnt[:n], oc):
            lines.append(f"level {l} cell counts differ: gpu {cnt[:n].tolist()} oracle {oc.tolist()}")
            break
    ng, no = len(kg), len(ko)
    lines.append(f"n gpu {ng} oracle {no}")
    m = min(ng, no)
    if m:
        diff = np.nonzero((kg[:m].view(np.uint8).reshape(m, 28) != ko[:m].view(np.uint8).reshape(m, 28)).any(axis=1))[0]
        if len(diff):
            i = diff[0]
            lines.append(f"first differing keypoint {i}: gpu {kg[i]} oracle {ko[i]}")
    return "\n".join(lines)


def _check_frame(ext, ora, img):
    kg, dg = ext(img)
    ko, do = ora.extract(img)
    if len(kg) != len(ko) or kg.tobytes() != ko.tobytes():
        pytest.fail("keypoints differ\n" + _diagnose(ext, ora, img, kg, ko))
    if len(ko) == 0:
        assert dg is None
        return kg, dg
    if dg.tobytes() != do.tobytes():
        rows = np.nonzero((dg != do).any(axis=1))[0]
        pytest.fail(f"descriptors differ in {len(rows)} rows, first {rows[:5]}: kp {kg[rows[0]]}")
    return kg, dg


CONFIGS = [
    # (W, H, nfeatures) — BASELINE.json configs C1/C2, the reference init extractor, C4, C5
    (640, 480, 1000),
    (640, 480, 2000),
    (1241, 376, 2000),
    (1280, 720, 2500),
]


@pytest.mark.parametrize("W,H,nf", CONFIGS)
def test_extract_parity_configs(W, H, nf):
    ext = orb.ORBextractor(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    ora = Oracle(nf, 1.2, 8, 1, 20)
    frames = orb.synth_stream(W, H, stream=3, first=0, count=3)
    for img in frames:
        _check_frame(ext, ora, img)


@pytest.mark.parametrize("W,H", [(320, 240), (641, 479), (752, 480), (161, 121)])
def test_extract_parity_odd_sizes(W, H):
    nf = 1000 if W >= 320 else 300
    ext = orb.ORBextractor(nf, 1.2, 8 if W >= 320 else 4, orb.FAST_SCORE, 20, device=0)
    ora = Oracle(nf, 1.2, 8 if W >= 320 else 4, 1, 20)
    for img in orb.synth_stream(W, H, stream=11, first=0, count=2):
        _check_frame(ext, ora, img)


@pytest.mark.parametrize("W,H,nf,nl,th", [(161, 121, 2000, 4, 20), (160, 120, 2000, 4, 7), (128, 96, 1500, 5, 12),
                                           (200, 150, 2000, 3, 20), (176, 144, 2000, 3, 7), (161, 121, 2000, 8, 7),
                                           (161, 121, 3000, 8, 20)])
def test_extract_parity_dense_cell_grids(W, H, nf, nl, th):
    """Many small cells: the ceil'd cell size makes the non-last cells' detection areas reach
    past maxBorder (ORBextractor.cc:572-597), so FAST runs beyond h-16 / w-16 there and the
    rBRIEF samples of such keypoints reach past the 3-px descriptor ring into raw padding."""
    ext = orb.ORBextractor(nf, 1.2, nl, orb.FAST_SCORE, th, device=0)
    ora = Oracle(nf, 1.2, nl, 1, th)
    for img in orb.synth_stream(W, H, stream=17, first=0, count=2):
        _check_frame(ext, ora, img)


@pytest.mark.parametrize("kind", [orb.SYN_FLAT, orb.SYN_LOWTEX, orb.SYN_NOISE])
def test_extract_parity_edge_frames(kind):
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    ora = Oracle(1000, 1.2, 8, 1, 20)
    img = orb.synth_special(kind, 640, 480, seed=5)
    kg, dg = _check_frame(ext, ora, img)
    if kind == orb.SYN_FLAT:
        assert len(kg) == 0 and dg is None  # _descriptors.release() path


def test_extract_parity_fast_thresholds():
    for th in (7, 12, 35):
        ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, th, device=0)
        ora = Oracle(1000, 1.2, 8, 1, th)
        _check_frame(ext, ora, orb.synth_stream(640, 480, stream=21, count=1)[0])


@pytest.mark.parametrize("W,H", [(640, 480), (1241, 376), (161, 121)])
def test_pyramid_and_descriptor_image_parity(W, H):
    """Every pyramid level (padded) and every descriptor image (blurred ROI + the raw ring
    rBRIEF can reach) against the oracle's ComputePyramid / GaussianBlur restatement."""
    nl = 8 if W >= 320 else 4
    ext = orb.ORBextractor(1000 if W >= 320 else 300, 1.2, nl, orb.FAST_SCORE, 20, device=0)
    ora = Oracle(1000 if W >= 320 else 300, 1.2, nl, 1, 20)
    img = orb.synth_stream(W, H, stream=13, count=1)[0]
    ext(img)
    ora.extract(img)
    lib = orb.hip_lib()
    for l in range(nl):
        w, h = ctypes.c_int(), ctypes.c_int()
        lib.orb_debug_level_image(ext._h, 0, l, None, ctypes.byref(w), ctypes.byref(h))
        w, h = w.value, h.value
        g = np.empty((h + 32, w + 32), np.uint8)
        lib.orb_debug_level_image(ext._h, 0, l, g.ctypes.data_as(ctypes.c_void_p), None, None)
        o = ora.level_image(l)
        assert np.array_equal(g, o), f"level {l} pyramid differs at {np.argwhere(g != o)[:5]}"
        bl = np.empty((h + 32, w + 32), np.uint8)
        lib.orb_debug_blur_image(ext._h, 0, l, bl.ctypes.data_as(ctypes.c_void_p))
        ob = np.empty((h, w), np.uint8)
        if ora.L.oracle_level_blurred(ora.h, l, ob.ctypes.data_as(ctypes.c_void_p)) == 0:
            assert np.array_equal(bl[16:16 + h, 16:16 + w], ob), f"level {l} blur differs"
        ring = np.zeros_like(bl, bool)
        ring[14:h + 18, 14:w + 18] = True
        ring[16:16 + h, 16:16 + w] = False
        assert np.array_equal(bl[ring], o[ring]), f"level {l} descriptor-image padding differs"


def test_empty_image_returns_untouched():
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    assert ext(np.zeros((0, 0), np.uint8)) == (None, None)


def test_batch_device_equals_single():
    import torch

    B, W, H = 6, 640, 480
    frames = orb.synth_stream(W, H, stream=2, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    kps, desc, counts = ext.extract_batch_device(d)
    torch.cuda.synchronize()
    kps, desc, counts = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    ora = Oracle(1000, 1.2, 8, 1, 20)
    for b in range(B):
        ko, do = ora.extract(frames[b])
        n = counts[b]
        assert n == len(ko)
        assert kps[b, :n].tobytes() == ko.tobytes()
        assert desc[b, :n].tobytes() == do.tobytes()
    # host-batch entry point too
    outs = ext.extract_batch(frames)
    for b in range(B):
        assert outs[b][0].tobytes() == kps[b, : counts[b]].tobytes()


def test_phase_split_equals_whole():
    """orb_extract_set_phases: pyramid (1) then the rest (2), with another batch's pyramid and
    extraction in between on a second extractor, is bit-identical to one mask-3 launch."""
    import torch

    B, W, H = 4, 640, 480
    frames = orb.synth_stream(W, H, stream=3, first=0, count=B)
    other = orb.synth_stream(W, H, stream=4, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    ext2 = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d, d2 = torch.from_numpy(frames).cuda(), torch.from_numpy(other).cuda()
    whole = [t.clone() for t in ext.extract_batch_device(d)]
    ext.set_phases(1)
    ext.extract_batch_device(d)
    ext2.extract_batch_device(d2)
    ext.set_phases(2)
    split = ext.extract_batch_device(d)
    ext.set_phases(3)
    torch.cuda.synchronize()
    n = whole[2].cpu().numpy()
    assert (split[2].cpu().numpy() == n).all()
    for b in range(B):
        assert split[0][b, : n[b]].cpu().numpy().tobytes() == whole[0][b, : n[b]].cpu().numpy().tobytes()
        assert split[1][b, : n[b]].cpu().numpy().tobytes() == whole[1][b, : n[b]].cpu().numpy().tobytes()
    # the host-buffer entry point ignores the phase mask
    ext.set_phases(1)
    outs = ext.extract_batch(frames)
    ext.set_phases(3)
    for b in range(B):
        assert outs[b][0].tobytes() == whole[0][b, : n[b]].cpu().numpy().tobytes()
    with pytest.raises(Exception):
        ext.set_phases(0)
    with pytest.raises(Exception):
        ext.set_phases(4)


# C2/C3, the reference init extractor nFeatures*2 (Tracking.cc:126, 217) at 640x480 / KITTI /
# 1280x720 (5000 kp: ~1086 level-0 keypoints, over k_match_init's LDS capacity -> the
# k_match_init_big fallback), C4, C5
@pytest.mark.parametrize("W,H,nf", [(640, 480, 1000), (640, 480, 2000), (1241, 376, 2000), (1241, 376, 4000),
                                    (1280, 720, 2500), (1280, 720, 5000)])
def test_search_for_initialization_parity(W, H, nf):
    ext = orb.ORBextractor(nf, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    frames = orb.synth_stream(W, H, stream=5, first=0, count=4)
    F = [orb.Frame.from_image(f, ext) for f in frames]
    matcher = orb.ORBmatcher(0.9, True)
    for a, b in [(0, 1), (1, 2), (0, 3)]:
        prev = np.ascontiguousarray(np.stack([F[a].mvKeys["x"], F[a].mvKeys["y"]], 1).astype(np.float32))
        prev_o = prev.copy()
        m12 = []
        n = matcher.SearchForInitialization(F[a], F[b], prev, m12, 100)
        no, m12o = search_for_initialization(F[a].mvKeys, F[a].mDescriptors, F[b].mvKeys, F[b].mDescriptors, W, H,
                                             prev_o, 0.9, True, 100)
        assert n == no
        assert np.array_equal(np.array(m12, np.int32), m12o)
        assert prev.tobytes() == prev_o.tobytes()
        assert n > 0
        # second call with the updated vbPrevMatched (Tracking::Initialize on the next frame)
        n2 = matcher.SearchForInitialization(F[a], F[b], prev, m12, 100)
        no2, m12o2 = search_for_initialization(F[a].mvKeys, F[a].mDescriptors, F[b].mvKeys, F[b].mDescriptors, W, H,
                                               prev_o, 0.9, True, 100)
        assert n2 == no2 and np.array_equal(np.array(m12, np.int32), m12o2)


@pytest.mark.parametrize("nnratio,checkOri,window", [(0.6, True, 10), (0.9, False, 50), (0.75, True, 200)])
def test_search_for_initialization_variants(nnratio, checkOri, window):
    W, H = 640, 480
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0)
    frames = orb.synth_stream(W, H, stream=9, first=0, count=2)
    F = [orb.Frame.from_image(f, ext) for f in frames]
    prev = np.ascontiguousarray(np.stack([F[0].mvKeys["x"], F[0].mvKeys["y"]], 1).astype(np.float32))
    prev_o = prev.copy()
    m12 = []
    n = orb.ORBmatcher(nnratio, checkOri).SearchForInitialization(F[0], F[1], prev, m12, window)
    no, m12o = search_for_initialization(F[0].mvKeys, F[0].mDescriptors, F[1].mvKeys, F[1].mDescriptors, W, H,
                                         prev_o, nnratio, checkOri, window)
    assert n == no and np.array_equal(np.array(m12, np.int32), m12o)


def test_match_batch_device_parity():
    import torch

    B, W, H = 8, 640, 480
    frames = orb.synth_stream(W, H, stream=4, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.FAST_SCORE, 20, device=0, max_batch=B)
    d = torch.from_numpy(frames).cuda()
    kps, desc, counts = ext.extract_batch_device(d)
    f1 = torch.arange(0, B - 1, dtype=torch.int32, device="cuda")
    f2 = f1 + 1
    m12, nm = orb.ORBmatcher(0.9, True).search_for_initialization_batch_device(kps, desc, counts, f1, f2, W, H, 100)
    torch.cuda.synchronize()
    kps_h, desc_h, cnt = kps.cpu().numpy(), desc.cpu().numpy(), counts.cpu().numpy()
    m12, nm = m12.cpu().numpy(), nm.cpu().numpy()
    for p in range(B - 1):
        n1, n2 = cnt[p], cnt[p + 1]
        k1 = orb.keypoints_from_bytes(kps_h[p], n1)
        k2 = orb.keypoints_from_bytes(kps_h[p + 1], n2)
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        no, m12o = search_for_initialization(k1, desc_h[p, :n1], k2, desc_h[p + 1, :n2], W, H, prev, 0.9, True, 100)
        assert nm[p] == no
        assert np.array_equal(m12[p, :n1], m12o)


@pytest.mark.parametrize("W,H,nf,th", [(640, 480, 1000, 20), (1241, 376, 2000, 20), (320, 240, 500, 12),
                                       (161, 121, 2000, 7)])
def test_extract_parity_harris_score(W, H, nf, th):
    """scoreType = HARRIS_SCORE (ORBextractor.cc:616-620): Harris responses (float) drive both
    retainBest passes and land in KeyPoint::response."""
    ext = orb.ORBextractor(nf, 1.2, 8, orb.HARRIS_SCORE, th, device=0)
    ora = Oracle(nf, 1.2, 8, 0, th)
    for img in orb.synth_stream(W, H, stream=11, first=0, count=2):
        kg, _ = _check_frame(ext, ora, img)
        assert len(kg) and not np.all(kg["response"] == np.round(kg["response"]))  # float responses


@pytest.mark.parametrize("kind", [orb.SYN_LOWTEX, orb.SYN_NOISE])
def test_extract_parity_harris_edge_frames(kind):
    ext = orb.ORBextractor(1000, 1.2, 8, orb.HARRIS_SCORE, 20, device=0)
    ora = Oracle(1000, 1.2, 8, 0, 20)
    _check_frame(ext, ora, orb.synth_special(kind, 640, 480, seed=5))


def test_harris_batch_device_equals_single():
    import torch

    W, H, B = 640, 480, 6
    frames = orb.synth_stream(W, H, stream=2, first=0, count=B)
    ext = orb.ORBextractor(1000, 1.2, 8, orb.HARRIS_SCORE, 20, device=0, max_batch=B)
    cap = ext.max_keypoints
    d_k = torch.empty((B, cap, 28), dtype=torch.uint8, device="cuda")
    d_d = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_c = torch.empty((B,), dtype=torch.int32, device="cuda")
    ext.extract_batch_device(torch.from_numpy(frames).cuda(), d_k, d_d, d_c)
    torch.cuda.synchronize()
    ora = Oracle(1000, 1.2, 8, 0, 20)
    cnt = d_c.cpu().numpy()
    kh, dh = d_k.cpu().numpy(), d_d.cpu().numpy()
    for b in range(B):
        ko, do = ora.extract(frames[b])
        assert cnt[b] == len(ko)
        assert kh[b, :cnt[b]].tobytes() == ko.tobytes()
        assert dh[b, :cnt[b]].tobytes() == do.tobytes()
