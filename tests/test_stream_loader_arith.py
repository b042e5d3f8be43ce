"""CPU check of k_pyr_stream's unaligned level-0 loads (load_unit16, orb_hip.hip).

A unit of 16 bytes at byte address p with nvalid valid bytes is rebuilt from the one or two
16-B-aligned blocks holding it: dwords w[d .. d+4] of the 32-B pair (d = (p & 15) >> 2), four
v_alignbyte funnel shifts by p & 3, bytes past nvalid cleared.  This restates that arithmetic
(v_alignbyte_b32(hi, lo, s) = low 32 bits of (hi:lo) >> 8s) and checks it against plain byte
slicing for every alignment and valid count, and that the second block is read only when it
holds a valid byte.  The GPU tests (test_gpu_pyramid_stream.py) check the kernel itself.
"""
import numpy as np


def alignbyte(hi, lo, s):
    return ((((int(hi) << 32) | int(lo)) >> (8 * s)) & 0xFFFFFFFF)


def load_unit16(mem, p, nvalid):
    sh, need = p & 15, min(nvalid, 16)
    base = p - sh
    second = sh + need > 16
    blocks = mem[base:base + 16].tobytes() + mem[base + (16 if second else 0):base + (32 if second else 16)].tobytes()
    w = np.frombuffer(blocks, "<u4")
    d, bs = sh >> 2, sh & 3
    s = [int(w[d + j]) for j in range(5)]
    o = [alignbyte(s[j + 1], s[j], bs) for j in range(4)]
    if need < 16:
        for q in range(4):
            nb = min(max(need - 4 * q, 0), 4)
            o[q] &= 0xFFFFFFFF if nb == 4 else (1 << (8 * nb)) - 1
    return np.array(o, "<u4").tobytes(), second


def test_funnel_shift_matches_bytes():
    rng = np.random.default_rng(0)
    mem = rng.integers(0, 256, 256, dtype=np.uint8)
    for p in range(16, 80):
        for nvalid in range(1, 21):
            got, second = load_unit16(mem, p, nvalid)
            need = min(nvalid, 16)
            want = mem[p:p + need].tobytes() + bytes(16 - need)
            assert got == want, (p, nvalid)
            # the second block is touched only when it holds one of the unit's valid bytes
            assert second == ((p + need - 1) // 16 != p // 16)


def test_row_end_never_reads_past_last_valid_block():
    # a 1241-byte row ending the buffer: the last unit's blocks stay inside the allocation
    W = 1241
    for r in range(4):
        row = r * W
        end = 4 * W
        for u in range((W + 15) // 16):
            p, nvalid = row + 16 * u, W - 16 * u
            sh, need = p & 15, min(nvalid, 16)
            last_block = p - sh + (16 if sh + need > 16 else 0)
            assert last_block < end and last_block <= p + need - 1
