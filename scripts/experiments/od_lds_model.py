#!/usr/bin/env python3
"""LDS bank-conflict model of one k_orient_desc keypoint wave, per access site (analysis
harness, CPU only).  Replays the kernel's LDS addresses (orb_hip.hip k_orient_desc: window
stores, IC_Angle reads, row-pass A reads and sum stores, rBRIEF column-pass reads) through the
gfx950 banking rules of MI355X_MICROARCH.md §LDS (lane groups per instruction, bank = dword
mod 32 or 64, each extra distinct address on a bank within a group = one extra cycle) for
keypoints at random window alignments and angles, and prints the mean extra (conflict) cycles
per wave per site -- the per-site split of SQ_LDS_BANK_CONFLICT.
Usage: od_lds_model.py [n_keypoints]"""
import math
import pathlib
import re
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
OD_WP, OD_HN, OD_WR, HALF = 64, 56, 21, 15
KOD = (0, 16, 28)


def groups(kind):
    if kind in ("b32", "w32", "read2"):
        return [list(range(0, 32)), list(range(32, 64))], 32
    if kind == "b128":
        g = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32))]
        g += [[x + 32 for x in gg] for gg in g]
        return g, 64
    if kind == "w128":
        return [list(range(8 * k, 8 * k + 8)) for k in range(8)], 32
    raise ValueError(kind)


def extra_cycles(kind, dwords):
    """dwords[lane] = list of dword addresses the lane touches in this access."""
    gs, nb = groups(kind)
    extra = 0
    for g in gs:
        banks = {}
        for ln in g:
            for d in dwords[ln]:
                banks.setdefault(d % nb, set()).add(d)
        worst = max(len(v) for v in banks.values()) if banks else 1
        extra += worst - 1
    return extra


def pattern():
    s = (ROOT / "orbslam_jpminipc_amd/csrc/pattern31.inc").read_text()
    body = s[s.index("{") + 1: s.index("}")]
    v = [int(x) for x in re.findall(r"-?\d+", body)]
    return np.array(v[:1024], np.float32).reshape(512, 2)


def wave(rng, pat):
    site = {}
    # window stores: 3 x ds_write_b128, unit i of lane + 64 j at byte 16 i (64-B rows)
    e = 0
    for j in range(3):
        e += extra_cycles("w128", [[(16 * (ln + 64 * j)) // 4 + k for k in range(4)] for ln in range(64)])
    site["window_store"] = e
    # IC_Angle: 5 x ds_read_b32 of W32[(r + 6) * 16 + pd0 + c], n = lane + 64 j, r = n / 9
    x = int(rng.integers(16, 600))
    xa = (x - 5) & ~15
    pd0 = (x + 1 - xa) >> 2
    e = 0
    for j in range(5):
        e += extra_cycles("b32", [[(((ln + 64 * j) // 9) + OD_WR - HALF) * (OD_WP // 4) + pd0 + (ln + 64 * j) % 9]
                                  for ln in range(64)])
    site["ic_read"] = e
    # row pass A: 3 x ds_read_b128 of W4[(kOdRow[m] + r16) * 4 + h4]
    e = 0
    for m in range(3):
        e += extra_cycles("b128", [[((KOD[m] + (ln & 15)) * 4 + (ln >> 4)) * 4 + k for k in range(4)] for ln in range(64)])
    site["rowpass_read"] = e
    # row-pass sums: per (m, t) two dword stores q[16 t], q[16 t + 56] (tile 3 to q3)
    e = 0
    for m in range(3):
        for t in range(4):
            for half in (0, 1):
                dw = []
                for ln in range(64):
                    r16, h4 = ln & 15, ln >> 4
                    if t < 3:
                        base = (KOD[m] // 2 + 2 * h4) * OD_HN + r16 + 16 * t
                    else:
                        q3 = 2 * h4 * OD_HN + r16 + (32 if r16 >= 8 else 48)
                        q3 += (8 * OD_HN if m >= 1 else 0) + (6 * OD_HN if m >= 2 else 0)
                        base = q3
                    dw.append([base + half * OD_HN])
                e += extra_cycles("w32", dw)
    site["rowpass_store"] = e
    # rBRIEF column pass: per sample q, ds_read2_b32 (0, 56) + (112, 168) at hq
    ang = float(rng.uniform(0, 360)) * math.pi / 180
    a, b = math.cos(ang), math.sin(ang)
    o0 = x - 5 - xa
    e = 0
    for q in range(8):
        dws = [[], [], [], []]
        for ln in range(64):
            px, py = pat[8 * ln + q]
            dy = int(np.rint(px * b + py * a))
            dx = int(np.rint(px * a - py * b))
            r0, hc = dy + 18, dx + 18
            base = (r0 >> 1) * OD_HN + hc + o0
            for k in range(4):
                dws[k].append([base + k * OD_HN])
        e += extra_cycles("read2", dws[0]) + extra_cycles("read2", dws[1])
        e += extra_cycles("read2", dws[2]) + extra_cycles("read2", dws[3])
    site["sample_read"] = e
    return site


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    rng = np.random.default_rng(1)
    pat = pattern()
    acc = {}
    for _ in range(n):
        for k, v in wave(rng, pat).items():
            acc[k] = acc.get(k, 0) + v
    tot = sum(acc.values())
    print(f"modelled LDS bank-conflict cycles per keypoint wave ({n} random keypoints): {tot / n:.1f}")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:14s} {v / n:6.1f}  ({100 * v / tot:.0f} %)")


if __name__ == "__main__":
    main()
