"""TEST INFRASTRUCTURE: synthetic DBoW2 vocabularies and a pure-Python restatement of
TemplatedVocabulary::transform (reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:
1126-1194, 1217-1259; BowVector.cpp:34-84; FeatureVector.cpp:31-45).

The reference ships no vocabulary (Data/ORBvoc.txt is absent), so test
vocabularies are built here: a hierarchical k-medians over real ORB descriptors, the way
DBoW2's HKmeansStep shapes a tree (children of a node contiguous, parents before children),
with centres = FORB::meanValue (bitwise majority, FORB.cpp:28-77).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from oracle_lib import _p, lib

POPCNT8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """FORB::distance for every pair (rows of a) x (rows of b)."""
    return POPCNT8[np.bitwise_xor(a[:, None, :], b[None, :, :])].sum(axis=2)


def mean_value(d: np.ndarray) -> np.ndarray:
    """FORB::meanValue: bit set iff set in at least ceil(N/2) descriptors (FORB.cpp:28-77)."""
    if len(d) == 1:
        return d[0].copy()
    bits = np.unpackbits(d, axis=1, bitorder="big").sum(axis=0)
    n2 = len(d) // 2 + len(d) % 2
    return np.packbits((bits >= n2).astype(np.uint8), bitorder="big")


def build_vocabulary(descs: np.ndarray, k: int = 10, L: int = 4, seed: int = 0, iters: int = 2,
                     stop_frac: float = 0.0, shallow_leaves: bool = False):
    """(parent, is_leaf, desc, weight) arrays of a k-ary tree of depth <= L over `descs`."""
    rng = np.random.default_rng(seed)
    parent, is_leaf, desc, weight = [], [], [], []

    def add(p, leaf, d, w):
        parent.append(p)
        is_leaf.append(1 if leaf else 0)
        desc.append(np.asarray(d, np.uint8))
        weight.append(w)
        return len(parent)  # node id (root = 0)

    def split(members):
        m = descs[members]
        if len(m) <= k:
            return [np.array([i]) for i in range(len(m))], [m[i] for i in range(len(m))]
        centres = m[rng.choice(len(m), size=k, replace=False)]
        for _ in range(iters):
            lab = np.argmin(hamming_matrix(m, centres), axis=1)
            groups = [np.nonzero(lab == c)[0] for c in range(k)]
            centres = np.stack([mean_value(m[g]) if len(g) else centres[c] for c, g in enumerate(groups)])
        lab = np.argmin(hamming_matrix(m, centres), axis=1)
        groups = [np.nonzero(lab == c)[0] for c in range(k)]
        keep = [c for c in range(k) if len(groups[c])]
        return [groups[c] for c in keep], [centres[c] for c in keep]

    todo = [(0, np.arange(len(descs)), 0)]
    while todo:
        nid, members, depth = todo.pop(0)
        groups, centres = split(members)
        kids = []
        for g, c in zip(groups, centres):
            leaf = depth + 1 == L or len(g) <= 1 or (shallow_leaves and depth + 1 >= 2 and rng.random() < 0.2)
            w = 0.0
            if leaf:
                w = 0.0 if rng.random() < stop_frac else float(rng.uniform(0.05, 4.0))
            cid = add(nid, leaf, c, w)
            if not leaf:
                kids.append((cid, members[g], depth + 1))
        todo.extend(kids)
    return (np.array(parent, np.int32), np.array(is_leaf, np.uint8), np.stack(desc).astype(np.uint8),
            np.array(weight, np.float64))


def random_vocabulary(k: int, L: int, seed: int = 0, bits: int = 256):
    """Complete k-ary tree of depth L with random node descriptors (few set bits when
    bits < 256: many distance ties)."""
    rng = np.random.default_rng(seed)
    parent, leaf = [], []
    level = [0]
    nid = 0
    for depth in range(1, L + 1):
        nxt = []
        for p in level:
            for _ in range(k):
                nid += 1
                parent.append(p)
                leaf.append(1 if depth == L else 0)
                nxt.append(nid)
        level = nxt
    n = len(parent)
    if bits >= 256:
        desc = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    else:
        desc = np.zeros((n, 32), np.uint8)
        for i in range(n):
            for b in rng.choice(256, size=bits, replace=False):
                desc[i, b // 8] |= np.uint8(1 << (b % 8))
    weight = np.where(np.array(leaf) > 0, rng.uniform(0.0, 3.0, size=n), 0.0)
    return np.array(parent, np.int32), np.array(leaf, np.uint8), desc, weight


# ---- pure-Python restatement ---------------------------------------------------------------
class PyVocabulary:
    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        self.k, self.L, self.scoring, self.weighting = k, L, scoring, weighting
        n = len(parent)
        self.children = [[] for _ in range(n + 1)]
        self.word = [0] * (n + 1)
        self.weight = [0.0] * (n + 1)
        self.desc = [np.zeros(32, np.uint8)] + [np.asarray(d, np.uint8) for d in desc]
        self.nwords = 0
        for i in range(n):
            self.children[int(parent[i])].append(i + 1)
            self.weight[i + 1] = float(weight[i])
            if is_leaf[i]:
                self.word[i + 1] = self.nwords
                self.nwords += 1

    def transform1(self, f, levelsup):
        nid_level = self.L - levelsup
        nid = 0 if nid_level <= 0 else None
        node, level = 0, 0
        while True:
            level += 1
            ch = self.children[node]
            best, bd = ch[0], int(POPCNT8[np.bitwise_xor(f, self.desc[ch[0]])].sum())
            for c in ch[1:]:
                d = int(POPCNT8[np.bitwise_xor(f, self.desc[c])].sum())
                if d < bd:
                    best, bd = c, d
            node = best
            if level == nid_level:
                nid = node
            if not self.children[node]:
                break
        return self.word[node], self.weight[node], (node if nid is None else nid)

    def transform(self, feats, levelsup):
        bow, fv = {}, {}
        if self.nwords == 0:
            return bow, fv
        tf = self.weighting in (0, 1)
        must = self.scoring != 5
        for i, f in enumerate(feats):
            w_id, w, nid = self.transform1(f, levelsup)
            if w > 0:
                if tf:
                    bow[w_id] = bow[w_id] + w if w_id in bow else w
                elif w_id not in bow:
                    bow[w_id] = w
                fv.setdefault(nid, []).append(i)
        keys = sorted(bow)
        if tf and bow and not must:
            nd = float(len(bow))
            for key in keys:
                bow[key] /= nd
        if must:
            norm = 0.0
            if self.scoring == 1:
                for key in keys:
                    norm = math.fma(bow[key], bow[key], norm) if hasattr(math, "fma") else _fma(bow[key], bow[key], norm)
                norm = math.sqrt(norm)
            else:
                for key in keys:
                    norm += abs(bow[key])
            if norm > 0.0:
                for key in keys:
                    bow[key] /= norm
        return {key: bow[key] for key in keys}, {key: fv[key] for key in sorted(fv)}


def _fma(a, b, c):
    """Exactly rounded a*b + c for doubles (Python < 3.13 has no math.fma)."""
    from fractions import Fraction

    return float(Fraction(a) * Fraction(b) + Fraction(c))


# ---- oracle bindings ------------------------------------------------------------------------
def _bind(L):
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.oracle_vocabulary_load_text.restype = vp
    L.oracle_vocabulary_load_text.argtypes = [ctypes.c_char_p]
    L.oracle_vocabulary_create.restype = vp
    L.oracle_vocabulary_create.argtypes = [i, i, i, i, i, vp, vp, vp, vp]
    L.oracle_vocabulary_destroy.argtypes = [vp]
    L.oracle_vocabulary_info.argtypes = [vp, vp]
    L.oracle_vocabulary_transform_one.argtypes = [vp, vp, i, vp, vp, vp]
    L.oracle_vocabulary_transform.argtypes = [vp, vp, i, i, vp, vp, ctypes.POINTER(i), vp, vp, vp, ctypes.POINTER(i)]


class OracleVocabulary:
    """CPU restatement (oracle/orb_oracle_voc.cpp)."""

    def __init__(self, handle):
        self.L = lib()
        if not getattr(self.L, "_voc_bound", False):
            _bind(self.L)
            self.L._voc_bound = True
        if not handle:
            raise ValueError("oracle vocabulary construction failed")
        self.h = handle

    @classmethod
    def create(cls, k, Ld, scoring, weighting, parent, is_leaf, desc, weight):
        L = lib()
        if not getattr(L, "_voc_bound", False):
            _bind(L)
            L._voc_bound = True
        parent = np.ascontiguousarray(parent, np.int32)
        leaf = np.ascontiguousarray(is_leaf, np.uint8)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        w = np.ascontiguousarray(weight, np.float64)
        return cls(L.oracle_vocabulary_create(k, Ld, scoring, weighting, len(parent), _p(parent), _p(leaf), _p(d),
                                              _p(w)))

    @classmethod
    def load_text(cls, path):
        L = lib()
        if not getattr(L, "_voc_bound", False):
            _bind(L)
            L._voc_bound = True
        h = L.oracle_vocabulary_load_text(str(path).encode())
        return cls(h) if h else None

    def __del__(self):
        try:
            self.L.oracle_vocabulary_destroy(self.h)
        except Exception:
            pass

    def info(self):
        out = np.zeros(6, np.int32)
        self.L.oracle_vocabulary_info(self.h, _p(out))
        return out

    def transform_one(self, d, levelsup):
        d = np.ascontiguousarray(d, np.uint8)
        w = np.zeros(1, np.uint32)
        wt = np.zeros(1, np.float64)
        n = np.zeros(1, np.uint32)
        assert self.L.oracle_vocabulary_transform_one(self.h, _p(d), int(levelsup), _p(w), _p(wt), _p(n)) == 0
        return int(w[0]), float(wt[0]), int(n[0])

    def transform(self, desc, levelsup):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        bw = np.zeros(max(n, 1), np.uint32)
        bv = np.zeros(max(n, 1), np.float64)
        fn = np.zeros(max(n, 1), np.uint32)
        fo = np.zeros(n + 1, np.int32)
        ff = np.zeros(max(n, 1), np.int32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        assert self.L.oracle_vocabulary_transform(self.h, _p(d), n, int(levelsup), _p(bw), _p(bv), ctypes.byref(nb),
                                                  _p(fn), _p(fo), _p(ff), ctypes.byref(nf)) == 0
        nb, nf = nb.value, nf.value
        return bw[:nb].copy(), bv[:nb].copy(), fn[:nf].copy(), fo[:nf + 1].copy(), ff[:fo[nf]].copy()
