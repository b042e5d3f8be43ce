"""MapPoint::ComputeDistinctiveDescriptors (reference src/MapPoint.cc:185-250): the oracle
against a numpy restatement on the CPU, and the HIP kernel against the oracle on the GPU."""
import ctypes

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd.mappoint import compute_distinctive_descriptors
from oracle_lib import Oracle, _p, lib
from vocab_util import POPCNT8


def _oracle(offsets, desc, usable):
    L = lib()
    L.oracle_compute_distinctive_descriptors.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5
    M = len(offsets) - 1
    best = np.full(M, -7, np.int32)
    out = np.zeros((M, 32), np.uint8)
    off = np.ascontiguousarray(offsets, np.int32)
    d = np.ascontiguousarray(desc, np.uint8)
    u = None if usable is None else np.ascontiguousarray(usable, np.uint8)
    assert L.oracle_compute_distinctive_descriptors(M, _p(off), _p(d), _p(u), _p(best), _p(out)) == 0
    return best, out


def _numpy(offsets, desc, usable):
    best = []
    for m in range(len(offsets) - 1):
        rows = [r for r in range(offsets[m], offsets[m + 1]) if usable is None or usable[r]]
        if not rows:
            best.append(-1)
            continue
        D = POPCNT8[np.bitwise_xor(desc[rows][:, None, :], desc[rows][None, :, :])].sum(axis=2)
        med = np.sort(D, axis=1)[:, (len(rows) - 1) // 2]
        best.append(rows[int(np.argmin(med))])  # argmin: first minimum
    return np.array(best, np.int32)


def _case(seed, sizes, frac_bad=0.2, near=True):
    rng = np.random.default_rng(seed)
    descs = Oracle(1000, 1.2, 8, 1, 20).extract(orb.synth_stream(640, 480, stream=50 + seed, count=1)[0])[1]
    rows, offsets = [], [0]
    for n in sizes:
        base = descs[rng.integers(len(descs))]
        for _ in range(n):
            d = base.copy()
            if near:  # observations of one point: a few flipped bits (many equal medians)
                for b in rng.choice(256, size=int(rng.integers(0, 12)), replace=False):
                    d[b // 8] ^= np.uint8(1 << (b % 8))
            else:
                d = descs[rng.integers(len(descs))]
            rows.append(d)
        offsets.append(len(rows))
    desc = np.stack(rows) if rows else np.zeros((0, 32), np.uint8)
    usable = (rng.random(len(rows)) > frac_bad).astype(np.uint8)
    return np.array(offsets, np.int32), desc, usable


SIZES = [1, 2, 3, 4, 5, 10, 0, 31, 64, 65, 130, 7, 2, 1]


@pytest.mark.parametrize("seed,near", [(0, True), (1, False), (2, True)])
def test_oracle_matches_numpy(seed, near):
    off, desc, usable = _case(seed, SIZES, near=near)
    for u in (usable, None):
        best, out = _oracle(off, desc, u)
        assert best.tolist() == _numpy(off, desc, u).tolist()
        for m, r in enumerate(best):
            if r >= 0:
                assert out[m].tobytes() == desc[r].tobytes()


def test_host_validation():
    with pytest.raises(orb.OrbError):
        compute_distinctive_descriptors([0, 3, 2], np.zeros((3, 32), np.uint8))  # decreasing offsets


@pytest.mark.gpu
@pytest.mark.parametrize("seed,near", [(0, True), (1, False), (3, True)])
def test_gpu_matches_oracle(seed, near):
    off, desc, usable = _case(seed, SIZES + [300, 1000], near=near)
    for u in (usable, None):
        cur = np.full((len(off) - 1, 32), 0xAB, np.uint8)
        best, out = compute_distinctive_descriptors(off, desc, u, current=cur)
        ob, oo = _oracle(off, desc, u)
        assert best.tolist() == ob.tolist()
        for m, r in enumerate(ob):
            assert out[m].tobytes() == (oo[m].tobytes() if r >= 0 else cur[m].tobytes())


@pytest.mark.gpu
def test_gpu_all_rows_bad_and_empty():
    off = np.array([0, 3, 3], np.int32)
    desc = np.arange(96, dtype=np.uint8).reshape(3, 32)
    best, out = compute_distinctive_descriptors(off, desc, np.zeros(3, np.uint8), current=np.ones((2, 32), np.uint8))
    assert best.tolist() == [-1, -1] and (out == 1).all()
    best, out = compute_distinctive_descriptors([0], np.zeros((0, 32), np.uint8))
    assert len(best) == 0
