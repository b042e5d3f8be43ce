"""CPU: the oracle's Frame::UndistortKeyPoints / ComputeImageBounds (oracle/orb_oracle_frame.cpp).

cv::undistortPoints is OpenCV 2.4 (cvUndistortPoints, imgproc/src/undistort.cpp), absent here:
parity against a real OpenCV binary is unpinned, like the other OpenCV primitives (DESIGN.md
§2).  What pins the restatement:
* an independent numpy restatement of the same published algorithm (float64 scalars, the same
  operation order), bit-exact against the oracle;
* the published distortion model itself: distorting a point with the Brown-Conrady forward model
  OpenCV documents (x_d = x (1 + k1 r^2 + k2 r^4) + 2 p1 x y + p2 (r^2 + 2 x^2), likewise y) and
  undistorting it returns the point (5 fixed iterations converge for moderate distortion);
* the reference's k1 == 0 branches (Frame.cc:291-295, 342-347).
"""
import numpy as np
import pytest

from oracle_lib import KEYPOINT_DTYPE, compute_image_bounds, undistort_keypoints, undistort_points

# (fx, fy, cx, cy), (k1, k2, p1, p2): a VGA ueye-like camera, KITTI-like, and a strong fisheye-ish one
CAMERAS = [
    ((458.654, 457.296, 367.215, 248.375), (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)),
    ((718.856, 718.856, 607.1928, 185.2157), (-0.2, 0.05, 0.001, -0.0005)),
    ((320.0, 320.0, 320.0, 240.0), (-0.35, 0.12, -0.002, 0.003)),
    ((500.0, 480.0, 300.5, 260.25), (0.15, -0.02, 0.0, 0.0)),
]


def np_undistort(xy, K4, d4):
    """numpy float64 restatement of cvUndistortPoints(src, dst, K, dist, NULL, K) (2.4)."""
    fx, fy, cx, cy = (np.float64(np.float32(v)) for v in K4)
    k = [np.float64(np.float32(v)) for v in d4] + [np.float64(0.0)] * 4
    ifx, ify = np.float64(1.0) / fx, np.float64(1.0) / fy
    out = np.empty_like(xy)
    two = np.float64(2.0)
    one = np.float64(1.0)
    for i, (px, py) in enumerate(xy):
        x0 = x = (np.float64(px) - cx) * ifx
        y0 = y = (np.float64(py) - cy) * ify
        for _ in range(5):
            r2 = x * x + y * y
            icdist = (one + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (one + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dX = two * k[2] * x * y + k[3] * (r2 + two * x * x)
            dY = k[2] * (r2 + two * y * y) + two * k[3] * x * y
            x = (x0 - dX) * icdist
            y = (y0 - dY) * icdist
        xx = fx * x + np.float64(0.0) * y + cx
        yy = np.float64(0.0) * x + fy * y + cy
        ww = one / (np.float64(0.0) * x + np.float64(0.0) * y + one)
        out[i] = (np.float32(xx * ww), np.float32(yy * ww))
    return out


def distort(xy, K4, d4):
    """Brown-Conrady forward model (float64), pixel in -> pixel out."""
    fx, fy, cx, cy = (float(v) for v in np.float32(K4))
    k1, k2, p1, p2 = (float(v) for v in np.float32(d4))
    x = (xy[:, 0] - cx) / fx
    y = (xy[:, 1] - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


@pytest.mark.parametrize("cam", range(len(CAMERAS)))
def test_oracle_equals_numpy_restatement(cam):
    K4, d4 = CAMERAS[cam]
    rng = np.random.default_rng(cam)
    xy = np.concatenate([rng.uniform(-50, 800, (3000, 2)),
                         np.array([[0, 0], [640, 0], [0, 480], [640, 480], K4[2:4]])]).astype(np.float32)
    got = undistort_points(xy, K4, d4)
    assert got.tobytes() == np_undistort(xy, K4, d4).tobytes()


@pytest.mark.parametrize("cam", [0, 1, 3])
def test_round_trip_through_the_forward_model(cam):
    K4, d4 = CAMERAS[cam]
    rng = np.random.default_rng(10 + cam)
    und = np.stack([rng.uniform(K4[2] - 250, K4[2] + 250, 2000), rng.uniform(K4[3] - 150, K4[3] + 150, 2000)], 1)
    dist = distort(und, K4, d4).astype(np.float32)
    back = undistort_points(dist, K4, d4).astype(np.float64)
    # fixed 5 iterations, not converged to float precision at the strongest corners
    assert np.abs(back - und).max() < 0.05, np.abs(back - und).max()


def test_k1_zero_is_a_copy_and_the_image_rectangle():
    rng = np.random.default_rng(3)
    kps = np.zeros(100, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(0, 640, 100)
    kps["y"] = rng.uniform(0, 480, 100)
    kps["octave"] = rng.integers(0, 8, 100)
    # k1 == 0 decides (Frame.cc:291), even with the other coefficients set
    d4 = (0.0, 0.1, 0.01, 0.01)
    assert undistort_keypoints(kps, CAMERAS[0][0], d4).tobytes() == kps.tobytes()
    assert compute_image_bounds(640, 480, CAMERAS[0][0], d4) == (0, 640, 0, 480)


def test_keypoints_keep_every_other_field():
    K4, d4 = CAMERAS[1]
    rng = np.random.default_rng(4)
    kps = np.zeros(64, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(0, 1241, 64)
    kps["y"] = rng.uniform(0, 376, 64)
    kps["size"] = 31
    kps["angle"] = rng.uniform(0, 360, 64)
    kps["response"] = rng.integers(20, 90, 64)
    kps["octave"] = rng.integers(0, 8, 64)
    kps["class_id"] = -1
    out = undistort_keypoints(kps, K4, d4)
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert out[f].tobytes() == kps[f].tobytes()
    xy = np.stack([kps["x"], kps["y"]], 1).astype(np.float32)
    assert np.stack([out["x"], out["y"]], 1).tobytes() == np_undistort(xy, K4, d4).tobytes()


def test_image_bounds_barrel_distortion():
    """Barrel distortion (k1 < 0) pulls the undistorted corners outward: the bounds grow past
    the image rectangle, floor / ceil of the corner coordinates (Frame.cc:335-338)."""
    K4, d4 = CAMERAS[0]
    b = compute_image_bounds(752, 480, K4, d4)
    c = np_undistort(np.array([[0, 0], [752, 0], [0, 480], [752, 480]], np.float32), K4, d4)
    assert b == (int(min(np.floor(c[0, 0]), np.floor(c[2, 0]))), int(max(np.ceil(c[1, 0]), np.ceil(c[3, 0]))),
                 int(min(np.floor(c[0, 1]), np.floor(c[1, 1]))), int(max(np.ceil(c[2, 1]), np.ceil(c[3, 1]))))
    assert b[0] < 0 and b[1] > 752 and b[2] < 0 and b[3] > 480
