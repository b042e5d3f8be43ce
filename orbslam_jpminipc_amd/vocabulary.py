"""ORBVocabulary on the GPU: DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>.

Mirrors the surface ORB-SLAM uses (reference include/ORBVocabulary.h and
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h): ``loadFromTextFile`` (1338-1424),
``transform(features, BowVector, FeatureVector, levelsup)`` (1126-1194) and the per-feature
``transform(feature, word_id, weight, nid, levelsup)`` (1217-1259), over the C ABI of
``include/orb_abi.h`` (csrc/orb_voc.hip).  BowVector comes back as a dict {word id: value} in
ascending word order (std::map order), FeatureVector as views.FeatureVector (CSR).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import check, hip_lib, ptr
from .views import FeatureVector

# BowVector.h:36-53
TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = 0, 1, 2, 3, 4, 5


class ORBVocabulary:
    """A vocabulary tree resident on one device."""

    def __init__(self, device: int = 0):
        self._lib = hip_lib()
        self._h = None
        self.device = int(device)

    # ---- construction ------------------------------------------------------------------
    def loadFromTextFile(self, filename: str) -> bool:
        """TemplatedVocabulary::loadFromTextFile; False when the file is not a vocabulary."""
        h = ctypes.c_void_p()
        st = self._lib.orb_vocabulary_load_text(str(filename).encode(), self.device, ctypes.byref(h))
        if st != 0:
            self.last_error = self._lib.orb_last_error().decode()
            return False
        self._replace(h)
        return True

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device: int = 0) -> "ORBVocabulary":
        """Node i + 1 <- (parent[i], is_leaf[i], desc[i], weight[i]): the text format's lines."""
        v = cls(device)
        parent = np.ascontiguousarray(np.asarray(parent, np.int32))
        leaf = np.ascontiguousarray(np.asarray(is_leaf, np.uint8))
        d = np.ascontiguousarray(np.asarray(desc, np.uint8).reshape(-1, 32))
        w = np.ascontiguousarray(np.asarray(weight, np.float64))
        n = len(parent)
        if not (len(leaf) == len(d) == len(w) == n):
            raise ValueError("node arrays differ in length")
        h = ctypes.c_void_p()
        check(v._lib.orb_vocabulary_create(int(k), int(L), int(scoring), int(weighting), n, ptr(parent), ptr(leaf),
                                           ptr(d), ptr(w), v.device, ctypes.byref(h)))
        v._replace(h)
        return v

    def _replace(self, h):
        self.close()
        self._h = h
        info = np.zeros(7, np.int32)
        check(self._lib.orb_vocabulary_info(self._h, ptr(info)))
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words, self.height = map(int, info)

    def close(self):
        if self._h:
            self._lib.orb_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # ---- TemplatedVocabulary accessors --------------------------------------------------
    def empty(self) -> bool:
        return self._h is None or self.n_words == 0

    def size(self) -> int:
        return 0 if self._h is None else self.n_words

    def getBranchingFactor(self) -> int:
        return self.k

    def getDepthLevels(self) -> int:
        return self.L

    def getScoringType(self) -> int:
        return self.scoring

    def getWeightingType(self) -> int:
        return self.weighting

    # ---- transform ----------------------------------------------------------------------
    def transform(self, features, levelsup: int = 4):
        """(BowVector dict, FeatureVector) of one frame's descriptors (N x 32 uint8)."""
        if self._h is None:
            return {}, FeatureVector([], [0], [])
        d = np.ascontiguousarray(np.asarray(features, np.uint8).reshape(-1, 32))
        n = len(d)
        bw = np.zeros(max(n, 1), np.uint32)
        bv = np.zeros(max(n, 1), np.float64)
        fn = np.zeros(max(n, 1), np.uint32)
        fo = np.zeros(n + 1, np.int32)
        ff = np.zeros(max(n, 1), np.int32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        check(self._lib.orb_vocabulary_transform(self._h, ptr(d), n, int(levelsup), ptr(bw), ptr(bv), ctypes.byref(nb),
                                                 ptr(fn), ptr(fo), ptr(ff), ctypes.byref(nf)))
        nb, nf = nb.value, nf.value
        bow = dict(zip(bw[:nb].tolist(), bv[:nb].tolist()))
        return bow, FeatureVector(fn[:nf], fo[:nf + 1], ff[:fo[nf]])

    def transform_features_device(self, d_desc, levelsup: int = 4, stream=None):
        """Per-descriptor (word id, weight, node at level L - levelsup) for (N, 32) device rows."""
        import torch

        n = int(d_desc.shape[0])
        dev = d_desc.device
        word = torch.empty((n,), dtype=torch.int32, device=dev)
        weight = torch.empty((n,), dtype=torch.float64, device=dev)
        node = torch.empty((n,), dtype=torch.int32, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.orb_vocabulary_transform_features_device(self._h, n, ptr(d_desc), int(levelsup), ptr(word),
                                                                 ptr(weight), ptr(node), ctypes.c_void_p(s.cuda_stream)))
        return word, weight, node

    def transform_batch_device(self, d_desc, d_counts, levelsup: int = 4, out: dict | None = None, stream=None):
        """Batched transform over extractor output: d_desc (B, cap, 32), d_counts (B,).

        Returns a dict of device tensors: feat_word / feat_weight / feat_node (B, cap),
        bow_words / bow_values (B, cap) with bow_n (B,), fv_nodes (B, cap), fv_offsets
        (B, cap + 1), fv_features (B, cap) with fv_n (B,).
        """
        import torch

        B, cap = int(d_desc.shape[0]), int(d_desc.shape[1])
        dev = d_desc.device
        if out is None:
            i32, u = torch.int32, dict(dtype=torch.int32, device=dev)
            out = {
                "feat_word": torch.empty((B, cap), **u), "feat_weight": torch.empty((B, cap), dtype=torch.float64,
                                                                                  device=dev),
                "feat_node": torch.empty((B, cap), **u), "bow_words": torch.empty((B, cap), **u),
                "bow_values": torch.empty((B, cap), dtype=torch.float64, device=dev),
                "bow_n": torch.empty((B,), dtype=i32, device=dev), "fv_nodes": torch.empty((B, cap), **u),
                "fv_offsets": torch.empty((B, cap + 1), **u), "fv_features": torch.empty((B, cap), **u),
                "fv_n": torch.empty((B,), dtype=i32, device=dev),
            }
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        o = out
        check(self._lib.orb_vocabulary_transform_batch_device(
            self._h, B, ptr(d_desc), ptr(d_counts), cap, int(levelsup), ptr(o["feat_word"]), ptr(o["feat_weight"]),
            ptr(o["feat_node"]), ptr(o["bow_words"]), ptr(o["bow_values"]), ptr(o["bow_n"]), ptr(o["fv_nodes"]),
            ptr(o["fv_offsets"]), ptr(o["fv_features"]), ptr(o["fv_n"]), ctypes.c_void_p(s.cuda_stream)))
        return out


def write_text(path, k, L, scoring, weighting, parent, is_leaf, desc, weight, weight_fmt: str = "%.17g") -> None:
    """Write a vocabulary in the format TemplatedVocabulary::saveToTextFile produces
    (TemplatedVocabulary.h:1429-1449).  The reference prints weights with the stream's
    default 6 significant digits; pass weight_fmt="%g" for that."""
    desc = np.asarray(desc, np.uint8).reshape(-1, 32)
    with open(path, "w") as f:
        f.write(f"{k} {L}  {scoring} {weighting}\n")
        for p, lf, d, w in zip(parent, is_leaf, desc, weight):
            f.write(f"{int(p)} {1 if lf else 0} " + " ".join(str(int(x)) for x in d) + "  " + (weight_fmt % w) + "\n")
