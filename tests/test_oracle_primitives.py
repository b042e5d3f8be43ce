"""The oracle's restatements of glibc / libstdc++ / OpenCV primitives vs the originals
that ARE available in this container (glibc libm, libstdc++), and self-consistency of the
ones that are not (OpenCV fastAtan2)."""
import ctypes
import pathlib
import subprocess

import numpy as np
import pytest

import orbslam_jpminipc_amd as orb
from oracle_lib import _p, lib

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_sincosf_restatement_matches_glibc_sample():
    """oracle_sinf/oracle_cosf (and the device copy) restate glibc 2.35's sinf/cosf; the full
    check over every float in [0, 2*pi] is scripts/check_trig_exhaustive.c (both bit-exact).
    Here: 2M random floats in the keypoint-angle domain, plus every 997th float."""
    libm = ctypes.CDLL("libm.so.6")
    libm.sinf.restype = ctypes.c_float
    libm.sinf.argtypes = [ctypes.c_float]
    libm.cosf.restype = ctypes.c_float
    libm.cosf.argtypes = [ctypes.c_float]
    L = lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 2 * np.pi, 20000).astype(np.float32),
                         np.arange(0, 0x40C90FDB, 997 * 4096, dtype=np.uint32).view(np.float32)])
    for x in xs[:: max(1, len(xs) // 20000)]:
        assert np.float32(L.oracle_sinf(float(x))).tobytes() == np.float32(libm.sinf(float(x))).tobytes()
        assert np.float32(L.oracle_cosf(float(x))).tobytes() == np.float32(libm.cosf(float(x))).tobytes()


def test_fast_atan2_properties():
    L = lib()
    f = L.oracle_fast_atan2
    assert f(0.0, 1.0) == 0.0
    assert abs(f(1.0, 0.0) - 90.0) < 1e-3
    assert abs(f(0.0, -1.0) - 180.0) < 1e-3
    assert abs(f(-1.0, 0.0) - 270.0) < 1e-3
    assert abs(f(1.0, 1.0) - 45.0) < 0.01
    assert f(0.0, 0.0) == 0.0  # IC_Angle of a flat patch
    rng = np.random.default_rng(2)
    for y, x in rng.integers(-3_000_000, 3_000_000, size=(2000, 2)):
        a = f(float(y), float(x))
        assert 0.0 <= a <= 360.0
        ref = np.degrees(np.arctan2(y, x)) % 360
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.01  # fastAtan2's polynomial is accurate to ~0.005 deg


def test_nth_element_replay_matches_libstdcxx():
    """The kernels' libstdc++ nth_element replay (csrc/nth_select.h, host instantiation in
    liborb_hip.so) against std::nth_element in the oracle, on tie-heavy FAST-score lists."""
    L = lib()
    hip = orb.hip_lib()
    rng = np.random.default_rng(7)
    for trial in range(600):
        n = int(rng.integers(1, 500))
        span = int(rng.integers(1, 30))
        scores = rng.integers(20, 20 + span, n).astype(np.uint32)
        if trial % 9 == 0:
            scores = np.sort(scores)
        keep = int(rng.integers(0, n + 1))
        packed = (scores << 24) | np.arange(n, dtype=np.uint32)
        a = packed.copy()
        hip.orb_debug_nth_element_u32(_p(a), n, keep)
        keys = scores.astype(np.float32)
        idx = np.arange(n, dtype=np.int32)
        L.oracle_nth_element_greater(_p(keys), _p(idx), n, keep)
        assert np.array_equal(a & 0xFFFFFF, idx.astype(np.uint32)), trial


def test_nth_element_native_check():
    """Compile and run tests/native/nth_check.cpp: orbsel:: vs libstdc++ including the
    depth-limited __heap_select branch."""
    exe = pathlib.Path("/tmp/orb_nth_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(ROOT / "tests/native/nth_check.cpp")],
                   check=True)
    r = subprocess.run([str(exe), "5000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
