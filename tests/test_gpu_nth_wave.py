"""The one-wave nth_element (csrc/nth_select.h: ballot-computed Hoare partitions) that k_select
uses for the per-level retainBest, against the sequential libstdc++ replay (itself checked
against std::nth_element in test_oracle_primitives.py) on tie-heavy score arrays."""
import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from orbslam_jpminipc_amd._native import ptr

pytestmark = pytest.mark.gpu


def _arrays():
    rng = np.random.default_rng(5)
    for n in [0, 1, 2, 3, 4, 5, 17, 63, 64, 65, 127, 128, 129, 240, 431, 1000, 2500, 6144]:
        for levels in (2, 8, 40, 256):
            scores = rng.integers(0, levels, size=n).astype(np.uint32)
            ident = rng.permutation(n).astype(np.uint32) & 0xFFFFFF
            yield (scores << 24) | ident
    yield np.full(300, 7 << 24, np.uint32) | np.arange(300, dtype=np.uint32)  # all equal
    yield (np.arange(500, dtype=np.uint32) % 256) << 24 | np.arange(500, dtype=np.uint32)  # sorted ramps


def test_wave_nth_element_equals_sequential_replay():
    lib = orb.hip_lib()
    rng = np.random.default_rng(6)
    checked = 0
    for a in _arrays():
        n = len(a)
        for nth in sorted({0, n // 2, max(n - 1, 0), int(rng.integers(0, n + 1)), n}):
            s = np.ascontiguousarray(a.copy())
            w = np.ascontiguousarray(a.copy())
            assert lib.orb_debug_nth_element_u32(ptr(s), n, nth) == 0
            assert lib.orb_debug_nth_element_wave_u32(ptr(w), n, nth, 0) == 0
            assert np.array_equal(s, w), (n, nth)
            checked += 1
    assert checked > 200
