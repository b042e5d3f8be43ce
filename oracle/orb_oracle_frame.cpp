// TEST INFRASTRUCTURE (CPU parity oracle; never part of the product path).
//
// Frame::UndistortKeyPoints (reference src/Frame.cc:289-319) and Frame::ComputeImageBounds
// (src/Frame.cc:321-349), with the OpenCV 2.4 primitive they call restated:
//   cv::undistortPoints(src, dst, K, distCoef, noArray(), K)
//     -> cvUndistortPoints(src, dst, K, dist, R = NULL, P = K)   (imgproc/src/undistort.cpp)
// as published in OpenCV 2.4: camera matrix and coefficients converted to double; with a
// distortion vector the correction is iterated a fixed 5 times (no convergence test); R = I,
// so RR = P * I = K exactly; the point is mapped back through RR and its homogeneous w; all in
// double, stored as float.  OpenCV is a baseline x86-64 build (no FMA contraction): this file
// is compiled -ffp-contract=off.  Parity unpinned against a real OpenCV 2.4 binary (none here),
// like the other OpenCV primitives.
//
// The reference's camera (Tracking.cc:52-70): K = eye(3) with fx, fy, cx, cy set
// (K = [fx 0 cx; 0 fy cy; 0 0 1]); mDistCoef = (k1, k2, p1, p2), CV_32F 4x1.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "orb_oracle.h"

namespace {

// cvUndistortPoints for one point (x, y), K = (fx, fy, cx, cy), k[8] = (k1, k2, p1, p2, 0...).
void undistort_one(const double A[3][3], const double RR[3][3], const double k[8], int iters, float xin, float yin,
                   float* xo, float* yo) {
    const double fx = A[0][0], fy = A[1][1], ifx = 1. / fx, ify = 1. / fy, cx = A[0][2], cy = A[1][2];
    double x = xin, y = yin, x0, y0;
    x0 = x = (x - cx) * ifx;
    y0 = y = (y - cy) * ify;
    for (int j = 0; j < iters; j++) {
        double r2 = x * x + y * y;
        double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
    double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
    double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
    *xo = (float)(xx * ww);
    *yo = (float)(yy * ww);
}

void camera(const float* K4, const float* dist4, double A[3][3], double RR[3][3], double k[8]) {
    std::memset(A, 0, 9 * sizeof(double));
    A[0][0] = K4[0];
    A[1][1] = K4[1];
    A[0][2] = K4[2];
    A[1][2] = K4[3];
    A[2][2] = 1;
    // RR = P * I with P = K: each entry a sum of products with 0 and 1, i.e. K exactly
    std::memcpy(RR, A, 9 * sizeof(double));
    for (int i = 0; i < 8; ++i) k[i] = i < 4 ? (double)dist4[i] : 0.0;
}

}  // namespace

extern "C" {

int oracle_undistort_points(const float* K4, const float* dist4, const float* xy, int n, float* out) {
    if (!K4 || !dist4 || n < 0 || (n && (!xy || !out))) return -1;
    double A[3][3], RR[3][3], k[8];
    camera(K4, dist4, A, RR, k);
    for (int i = 0; i < n; ++i) undistort_one(A, RR, k, 5, xy[2 * i], xy[2 * i + 1], &out[2 * i], &out[2 * i + 1]);
    return 0;
}

// Frame::UndistortKeyPoints: k1 == 0 -> mvKeysUn = mvKeys (Frame.cc:291-295), else every
// keypoint copied with its pt undistorted (Frame.cc:297-318).
int oracle_undistort_keypoints(const orb_keypoint_t* kps, int n, const float* K4, const float* dist4,
                               orb_keypoint_t* out) {
    if (!K4 || !dist4 || n < 0 || (n && (!kps || !out))) return -1;
    if (dist4[0] == 0.0) {
        std::memcpy(out, kps, sizeof(orb_keypoint_t) * (size_t)n);
        return 0;
    }
    double A[3][3], RR[3][3], k[8];
    camera(K4, dist4, A, RR, k);
    for (int i = 0; i < n; ++i) {
        out[i] = kps[i];
        undistort_one(A, RR, k, 5, kps[i].x, kps[i].y, &out[i].x, &out[i].y);
    }
    return 0;
}

// Frame::ComputeImageBounds (Frame.cc:321-349).
int oracle_compute_image_bounds(int cols, int rows, const float* K4, const float* dist4, orb_frame_bounds_t* b) {
    if (!K4 || !dist4 || !b) return -1;
    if (dist4[0] != 0.0) {
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float m[8];
        oracle_undistort_points(K4, dist4, c, 4, m);
        b->min_x = (int)std::min(std::floor(m[0]), std::floor(m[4]));
        b->max_x = (int)std::max(std::ceil(m[2]), std::ceil(m[6]));
        b->min_y = (int)std::min(std::floor(m[1]), std::floor(m[3]));
        b->max_y = (int)std::max(std::ceil(m[5]), std::ceil(m[7]));
    } else {
        b->min_x = 0;
        b->max_x = cols;
        b->min_y = 0;
        b->max_y = rows;
    }
    return 0;
}

}  // extern "C"
