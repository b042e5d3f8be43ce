"""GPU SearchForInitialization under match conflicts, ties and capacity edges.

k_match_init resolves the reference's sequential "a later query steals the slot"
rule (ORBmatcher.cc:640-680) in speculative batches; extractor
outputs rarely collide, so these frames are built to: descriptors drawn from a small
pool (every query wants the same few F2 slots), all-equal descriptors (every distance
ties), dense clusters, level-0 counts beyond the kernel's LDS capacity (the
k_match_init_big path) and empty frames.  Compared index-by-index with the oracle
(oracle/orb_oracle_match.cpp), on the first call and on the second call that reads the
updated vbPrevMatched.
"""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import search_for_initialization
from test_matcher_oracle import make_pair

pytestmark = pytest.mark.gpu

W, H = 640, 480


def _kps(rng, n, centre=None, spread=None, p0=0.8):
    k = np.zeros(n, orb.KEYPOINT_DTYPE)
    if centre is None:
        k["x"] = rng.uniform(0, W - 1, n)
        k["y"] = rng.uniform(0, H - 1, n)
    else:
        k["x"] = np.clip(rng.normal(centre[0], spread, n), 0, W - 1)
        k["y"] = np.clip(rng.normal(centre[1], spread, n), 0, H - 1)
    k["octave"] = np.where(rng.random(n) < p0, 0, rng.integers(1, 8, n))
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["size"] = 31
    k["response"] = rng.integers(1, 100, n)
    k["class_id"] = -1
    return k


def _flip(rng, d, nmax):
    d = d.copy()
    for r in range(len(d)):
        for b in rng.choice(256, int(rng.integers(0, nmax + 1)), replace=False):
            d[r, b // 8] ^= 1 << (b % 8)
    return d


def _run_both(k1, d1, k2, d2, nnratio=0.9, checkOri=True, window=100):
    F1, F2 = orb.Frame(k1, d1, W, H), orb.Frame(k2, d2, W, H)
    matcher = orb.ORBmatcher(nnratio, checkOri)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32)).reshape(len(k1), 2)
    prev_o = prev.copy()
    total = 0
    for _ in range(2):
        m12 = []
        n = matcher.SearchForInitialization(F1, F2, prev, m12, window)
        no, m12o = search_for_initialization(k1, d1, k2, d2, W, H, prev_o, nnratio, checkOri, window)
        assert n == no
        assert np.array_equal(np.array(m12, np.int32).reshape(-1), m12o)
        assert prev.tobytes() == prev_o.tobytes()
        total += n
    return total


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("n1,n2", [(600, 700), (1400, 1600), (3000, 2500)])
def test_sfi_random_pairs(seed, n1, n2):
    rng = np.random.default_rng(100 + seed)
    k1, d1, k2, d2 = make_pair(rng, n1, n2, W, H)
    assert _run_both(k1, d1, k2, d2) > 0


@pytest.mark.parametrize("n1,n2,p0", [(5800, 6000, 0.15), (8192, 8192, 0.12), (8192, 7000, 0.6)])
def test_sfi_large_capacity(n1, n2, p0):
    """Frames of up to 8192 keypoints (the ABI's limit): with few octave-0 keypoints the
    LDS body runs at that capacity (its per-keypoint LDS arrays sized by cap), with many
    the large-capacity body; neither may refuse the call (ORB_ENOTSUP)."""
    rng = np.random.default_rng(n1 + n2)
    k1, k2 = _kps(rng, n1, p0=p0), _kps(rng, n2, p0=p0)
    base = rng.integers(0, 256, (64, 32), dtype=np.uint8)  # shared bases: real candidates
    d1 = _flip(rng, base[rng.integers(0, 64, n1)], 12)
    d2 = _flip(rng, base[rng.integers(0, 64, n2)], 12)
    assert _run_both(k1, d1, k2, d2, 0.9, True, 40) > 0


@pytest.mark.parametrize("pool", [1, 3, 8, 32])
@pytest.mark.parametrize("nnratio,checkOri,window", [(0.9, True, 100), (1.0, False, 200), (0.6, True, 40)])
def test_sfi_descriptor_pool_conflicts(pool, nnratio, checkOri, window):
    """Every descriptor is one of `pool` bases plus 0-3 bit flips: queries in a window
    compete for the same best slots, so nearly every speculative batch has conflicts."""
    rng = np.random.default_rng(pool * 7 + int(window))
    base = rng.integers(0, 256, (pool, 32), dtype=np.uint8)
    k1 = _kps(rng, 900, (320, 240), 60)
    k2 = _kps(rng, 700, (320, 240), 60)
    d1 = _flip(rng, base[rng.integers(0, pool, 900)], 3)
    d2 = _flip(rng, base[rng.integers(0, pool, 700)], 3)
    _run_both(k1, d1, k2, d2, nnratio, checkOri, window)


@pytest.mark.parametrize("n1,n2", [(64, 64), (1000, 1000), (2000, 300)])
def test_sfi_all_equal_descriptors(n1, n2):
    """Every distance is 0, so best == second wherever a window holds two F2 keypoints and
    the strict ratio test (ORBmatcher.cc:660) rejects; only lone-candidate windows match."""
    rng = np.random.default_rng(n1 + n2)
    k1, k2 = _kps(rng, n1, (200, 200), 30), _kps(rng, n2, (200, 200), 30)
    d = rng.integers(0, 256, 32, dtype=np.uint8)
    d1, d2 = np.tile(d, (n1, 1)), np.tile(d, (n2, 1))
    _run_both(k1, d1, k2, d2, 0.9)
    _run_both(k1, d1, k2, d2, 1.0, False, 10)
    _run_both(k1, d1, k2, d2, 1.0, True, 3)


def test_sfi_single_f2_keypoint():
    """One F2 keypoint: every query's best slot is the same and second stays INT_MAX."""
    rng = np.random.default_rng(5)
    k1 = _kps(rng, 500, (320, 240), 20, p0=1.0)
    k2 = _kps(rng, 1, (320, 240), 1, p0=1.0)
    d2 = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    d1 = _flip(rng, np.tile(d2, (500, 1)), 40)
    assert _run_both(k1, d1, k2, d2, 0.9, True, 200) == 2  # one match per call


def test_sfi_empty_frames():
    rng = np.random.default_rng(6)
    k, d = _kps(rng, 50), rng.integers(0, 256, (50, 32), dtype=np.uint8)
    e, de = np.zeros(0, orb.KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8)
    assert _run_both(k, d, e, de) == 0
    assert _run_both(e, de, k, d) == 0
    # no level-0 keypoint in F1 (the reference skips octave > 0 queries)
    k0 = k.copy()
    k0["octave"] = 1
    assert _run_both(k0, d, k, d) == 0
