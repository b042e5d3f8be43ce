"""TEST INFRASTRUCTURE: seeded synthetic matcher scenes (frames, poses, MapPoints, vocabulary
buckets) for the ORBmatcher-family parity tests.  Geometry is built so that a good share of
the queries land on a true counterpart (small Hamming distance, consistent projection) and
the rest exercise every rejection branch: behind the camera, outside the image, outside the
distance band, viewing angle > 60 deg, taken targets, contention for one target, empty
windows, and long candidate lists that overflow the GPU's per-query top-8.
"""
from __future__ import annotations

import numpy as np

from orbslam_jpminipc_amd import KEYPOINT_DTYPE
from orbslam_jpminipc_amd.views import FeatureVector, MapPointSet, View, frame_scale_tables

W, H = 640, 480
CALIB = (520.9, 521.0, 325.1, 249.7)
NLEVELS = 8
SF, SIGMA2 = frame_scale_tables(NLEVELS, 1.2)


def rot(rng, max_angle=0.25):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    a = rng.uniform(-max_angle, max_angle)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return (np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K)


def keypoints(rng, n, clusters=10, spread=12.0, octave_p=None):
    k = np.zeros(n, KEYPOINT_DTYPE)
    centres = rng.uniform([20, 20], [W - 20, H - 20], (clusters, 2))
    near = rng.random(n) < 0.6
    xy = rng.uniform([0, 0], [W - 1, H - 1], (n, 2))
    c = centres[rng.integers(0, clusters, n)]
    xy[near] = np.clip(c[near] + rng.normal(0, spread, (near.sum(), 2)), 0, [W - 1, H - 1])
    k["x"], k["y"] = xy[:, 0], xy[:, 1]
    p = octave_p if octave_p is not None else 0.7 ** np.arange(NLEVELS)
    k["octave"] = rng.choice(NLEVELS, n, p=p / p.sum())
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["size"] = 31 * SF[k["octave"]]
    k["response"] = rng.integers(1, 100, n)
    k["class_id"] = -1
    return k


def descriptors(rng, n):
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


def perturb(rng, d, kmax):
    """Flip k ~ U[0, kmax] random bits per row."""
    d = d.copy()
    for i in range(len(d)):
        for b in rng.choice(256, int(rng.integers(0, kmax + 1)), replace=False):
            d[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def view(rng, n, R=None, t=None, **kw):
    return View(keypoints(rng, n, **kw), descriptors(rng, n), (0, W, 0, H), NLEVELS, 1.2, CALIB,
                R if R is not None else rot(rng), t if t is not None else rng.uniform(-0.5, 0.5, 3))


def backproject(V: View, u, v, z):
    """World points seen at pixel (u, v) with depth z from view V."""
    fx, fy, cx, cy = (float(c) for c in (V.fx, V.fy, V.cx, V.cy))
    u, v, z = np.broadcast_arrays(np.asarray(u, np.float64), np.asarray(v, np.float64), np.asarray(z, np.float64))
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    R = V.Rcw.astype(np.float64)
    t = V.tcw.astype(np.float64)
    return ((Xc - t) @ R).astype(np.float32)  # R^T (Xc - t)


def map_points_on(rng, T: View, m, pix_noise=1.5, kmax=70, bad_frac=0.15):
    """m MapPoints derived from T's keypoints (repeats allowed -> contention), plus a fraction
    of adversarial ones.  Returns (MapPointSet, source keypoint index per point)."""
    src = rng.integers(0, T.n, m)
    u = T.kps["x"][src] + rng.normal(0, pix_noise, m)
    v = T.kps["y"][src] + rng.normal(0, pix_noise, m)
    z = rng.uniform(1.0, 12.0, m)
    P = backproject(T, u, v, z)
    Ow = T.Ow.astype(np.float64)
    PO = P.astype(np.float64) - Ow
    dist = np.linalg.norm(PO, axis=1)
    nrm = PO / dist[:, None] + rng.normal(0, 0.1, (m, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    oct_ = T.kps["octave"][src]
    dmin = dist / (SF[oct_] * rng.uniform(0.85, 1.15, m))
    dmax = dmin * SF[NLEVELS - 1] * 1.2
    desc = perturb(rng, T.desc[src], kmax)
    # adversarial rows
    bad = rng.random(m) < bad_frac
    kind = rng.integers(0, 5, m)
    P[bad & (kind == 0)] = backproject(T, np.full((bad & (kind == 0)).sum(), 300.0),
                                       np.full((bad & (kind == 0)).sum(), 200.0),
                                       -rng.uniform(1, 5, (bad & (kind == 0)).sum()))  # behind
    sel = bad & (kind == 1)
    P[sel] = backproject(T, rng.uniform(-400, -10, sel.sum()), rng.uniform(0, H, sel.sum()), 5.0)  # outside
    sel = bad & (kind == 2)
    dmax[sel] = dist[sel] * 0.5  # beyond max distance
    sel = bad & (kind == 3)
    nrm[sel] = -nrm[sel]  # viewing angle > 60 deg
    sel = bad & (kind == 4)
    desc[sel] = descriptors(rng, sel.sum())  # no counterpart
    return MapPointSet(P, nrm, dmin.astype(np.float32), dmax.astype(np.float32), desc), src


def feature_vector(rng, n, n_nodes=60, node_ids=None, assign=None):
    """Random DBoW2 FeatureVector: each keypoint in one node, indices ascending per node."""
    ids = np.sort(rng.choice(100000, n_nodes, replace=False)) if node_ids is None else np.asarray(node_ids)
    a = rng.integers(0, len(ids), n) if assign is None else assign
    d = {}
    for i in range(n):
        d.setdefault(int(ids[a[i]]), []).append(i)
    return FeatureVector.from_dict(d), ids, a


def relative_pose(V1: View, V2: View):
    """R12, t12 with X1 = R12 X2 + t12 (camera 2 -> camera 1)."""
    R1, t1 = V1.Rcw.astype(np.float64), V1.tcw.astype(np.float64)
    R2, t2 = V2.Rcw.astype(np.float64), V2.tcw.astype(np.float64)
    R12 = R1 @ R2.T
    return R12, t1 - R12 @ t2


def fundamental12(V1: View, V2: View):
    """F12 with x1^T F12 x2 = 0 (ORB-SLAM's ComputeF12 convention), float32 row-major."""
    R12, t12 = relative_pose(V1, V2)
    K = np.array([[V1.fx, 0, V1.cx], [0, V1.fy, V1.cy], [0, 0, 1]], np.float64)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    Ki = np.linalg.inv(K)
    return (Ki.T @ tx @ R12 @ Ki).astype(np.float32)


def project(V: View, P):
    X = P.astype(np.float64) @ V.Rcw.astype(np.float64).T + V.tcw.astype(np.float64)
    return V.fx * X[:, 0] / X[:, 2] + V.cx, V.fy * X[:, 1] / X[:, 2] + V.cy, X[:, 2]


def two_views_of_points(rng, n_pts, n_extra=200, pix_noise=1.0, kmax=60):
    """Two keyframes observing common world points (+ extra random keypoints each).
    Returns V1, V2, P (world points), idx1, idx2 (keypoint index of point p in each view)."""
    R1, t1 = rot(rng, 0.1), rng.uniform(-0.2, 0.2, 3)
    R2, t2 = R1 @ rot(rng, 0.08), t1 + rng.uniform(-0.3, 0.3, 3)
    base = View(np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8), (0, W, 0, H), NLEVELS, 1.2, CALIB, R1, t1)
    u = rng.uniform(30, W - 30, n_pts)
    v = rng.uniform(30, H - 30, n_pts)
    P = backproject(base, u, v, rng.uniform(2, 8, n_pts))
    d0 = descriptors(rng, n_pts)
    views, idxs = [], []
    for R, t in ((R1, t1), (R2, t2)):
        V = View(np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8), (0, W, 0, H), NLEVELS, 1.2, CALIB, R, t)
        pu, pv, _ = project(V, P)
        k = keypoints(rng, n_pts + n_extra)
        perm = rng.permutation(n_pts + n_extra)
        idx = perm[:n_pts]
        k["x"][idx] = np.clip(pu + rng.normal(0, pix_noise, n_pts), 0, W - 1)
        k["y"][idx] = np.clip(pv + rng.normal(0, pix_noise, n_pts), 0, H - 1)
        k["angle"][idx] = (np.float32(rng.uniform(0, 360)) + rng.normal(0, 5, n_pts)).astype(np.float32) % 360
        dsc = descriptors(rng, n_pts + n_extra)
        dsc[idx] = perturb(rng, d0, kmax)
        views.append(View(k, dsc, (0, W, 0, H), NLEVELS, 1.2, CALIB, R, t))
        idxs.append(idx)
    return views[0], views[1], P, idxs[0], idxs[1]
