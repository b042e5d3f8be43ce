#!/usr/bin/env python3
"""Probe (experiment harness): SearchByBoW(KF, F) per call vs the oracle on random pairs with
small vocabulary nodes; prints the first differing output slot with its node's data."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import orbslam_jpminipc_amd as orb  # noqa: E402
from oracle_lib import OracleMatcher  # noqa: E402
import scenes as S  # noqa: E402
from test_gpu_matcher_family import _bow_pair  # noqa: E402

bad = 0
for seed in range(40):
    rng = np.random.default_rng(seed)
    V1, V2, fv1, fv2 = _bow_pair(rng)
    for chk in (False, True):
        g, o = orb.ORBmatcher(0.7, chk), OracleMatcher(0.7, chk)
        ng, og = g.SearchByBoW_KF_F(V1, None, fv1, V2, fv2)
        no, oo = o.SearchByBoW_KF_F(V1, None, fv1, V2, fv2)
        if ng != no or not np.array_equal(og, oo):
            bad += 1
            d = np.flatnonzero(og != oo)
            print(f"seed {seed} checkOri {chk}: n {ng} vs {no}; slots {d[:8].tolist()} gpu {og[d[:8]].tolist()} oracle {oo[d[:8]].tolist()}")
            if bad <= 2:
                # the node of the first differing F feature
                i2 = int(d[0])
                nodes2, off2, feat2 = fv2.nodes, fv2.offsets, fv2.features
                for a in range(len(nodes2)):
                    fs = feat2[off2[a]:off2[a + 1]].tolist()
                    if i2 in fs:
                        nid = nodes2[a]
                        a1 = int(np.searchsorted(fv1.nodes, nid))
                        q = fv1.features[fv1.offsets[a1]:fv1.offsets[a1 + 1]].tolist() if a1 < len(fv1.nodes) and fv1.nodes[a1] == nid else []
                        print("  node", int(nid), "queries", q, "candidates", fs)
                        D = np.array([[int(np.unpackbits(V1.desc[x] ^ V2.desc[y]).sum()) for y in fs] for x in q])
                        print("  dist\n", D)
                        print("  gpu out", og[fs].tolist(), "oracle", oo[fs].tolist())
                        break
print("bad", bad)
