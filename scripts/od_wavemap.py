#!/usr/bin/env python3
"""Map the differing descriptor rows of scripts/od_diag.py logs (640x480, 2000 kp, stream 3
frames 0-2) to k_orient_desc slots: the wave of the workgroup (slot % 4), the float4 pattern
load (test % 4) and the lanes (test // 4).  Usage: od_wavemap.py LOG..."""
import sys, re, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import orbslam_jpminipc_amd as orb
from oracle_lib import Oracle
NF = 2000
ora = Oracle(NF, 1.2, 8, 1, 20)
# nDesired per level (ORBextractor.cc:486-503)
f = 1.0 / 1.2
nd = NF * (1 - f) / (1 - f ** 8)
nDes = []
s = 0
for l in range(7):
    v = int(np.rint(nd)); nDes.append(v); s += v; nd *= f
nDes.append(max(NF - s, 0))
base = np.concatenate([[0], np.cumsum(nDes)[:-1]])
levels = {}
for fi, img in enumerate(orb.synth_stream(640, 480, stream=3, first=0, count=3)):
    k, _ = ora.extract(img)
    oc = np.bincount(k["octave"], minlength=8)
    levels[fi] = np.concatenate([[0], np.cumsum(oc)[:-1]])
from collections import Counter
for fn in sys.argv[1:]:
    waves = Counter(); qs = Counter(); lanes = Counter()
    fi = None
    for line in open(fn):
        m = re.match(r"frame (\d+) rep", line)
        if m: fi = int(m.group(1)); continue
        m = re.match(r"\s+row (\d+) kp .* level (\d+) tests \[(.*)\]", line)
        if m:
            r, l = int(m.group(1)), int(m.group(2))
            idx = r - levels[fi][l]
            k = base[l] + idx
            waves[k % 4] += 1
            t = [int(x) for x in m.group(3).split(",")]
            qs[tuple(sorted(set(x % 4 for x in t)))] += 1
            for x in t: lanes[x // 4] += 1
    print(fn, "waves", dict(waves), "q-sets", dict(qs), "lanes", sorted(lanes))
