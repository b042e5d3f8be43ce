// orb_frame.hip — the Frame-side keypoint geometry on the GPU (part of liborb_hip.so).
//
// Frame::UndistortKeyPoints (reference src/Frame.cc:289-319) and Frame::ComputeImageBounds
// (src/Frame.cc:321-349): between the extractor and the matchers, mvKeysUn is mvKeys with each
// point passed through cv::undistortPoints(pt, K, mDistCoef, noArray(), K), or a plain copy when
// k1 == 0 (Frame.cc:291-295).  OpenCV 2.4's cvUndistortPoints (imgproc/src/undistort.cpp) is
// restated in IEEE double, operation for operation (no contraction: the TU is built
// -ffp-contract=off; double division is correctly rounded on gfx950): normalise by the camera
// matrix, 5 fixed-point iterations of the distortion inverse, back through RR = K * I = K and its
// homogeneous w (= 1), rounded to float.
//
//   k_undistort  one thread per keypoint slot of a [B][cap] batch (slots past the frame's count
//                are left alone): 28-B record in, the same record with (x, y) replaced out.
//                HBM-bound, 56 B per keypoint.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>

#include "../../include/orb_abi.h"
#include "orb_internal.h"

namespace {

int fail(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }

#define FCHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// The reference camera (Tracking.cc:52-70): K = [fx 0 cx; 0 fy cy; 0 0 1], mDistCoef =
// (k1, k2, p1, p2); cvUndistortPoints widens both to double, k[4..7] = 0.
struct Camera {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2;
};

__device__ __forceinline__ void undistort_pt(const Camera& c, float xin, float yin, float* xo, float* yo) {
    const double k[8] = {c.k1, c.k2, c.p1, c.p2, 0.0, 0.0, 0.0, 0.0};
    const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    double x = xin, y = yin;
    const double x0 = x = (x - cx) * ifx;
    const double y0 = y = (y - cy) * ify;
#pragma unroll
    for (int j = 0; j < 5; j++) {  // iters = 5 whenever distortion coefficients are given
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = K: xx = fx x + 0 y + cx, yy = 0 x + fy y + cy, w = 1 / (0 x + 0 y + 1)
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *xo = (float)(xx * ww);
    *yo = (float)(yy * ww);
}

// kps and out may alias (the ABI allows d_kps_un == d_kps): no __restrict__ on them; each thread
// reads its record before writing the same slot.
__global__ void __launch_bounds__(256) k_undistort(const orb_keypoint_t* kps, const int32_t* __restrict__ counts,
                                                   int cap, int B, Camera cam, orb_keypoint_t* out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)B * cap) return;
    const int b = (int)(i / cap), k = (int)(i - (long long)b * cap);
    if (k >= counts[b]) return;
    orb_keypoint_t kp = kps[i];
    if (cam.k1 != 0.0f) undistort_pt(cam, kp.x, kp.y, &kp.x, &kp.y);
    out[i] = kp;
}

// Generic points: xy[2n] -> out[2n] (no k1 == 0 shortcut: cv::undistortPoints itself).
__global__ void __launch_bounds__(256) k_undistort_points(const float* __restrict__ xy, int n, Camera cam,
                                                          float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float x, y;
    undistort_pt(cam, xy[2 * i], xy[2 * i + 1], &x, &y);
    out[2 * i] = x;
    out[2 * i + 1] = y;
}

int camera_of(const float* K4, const float* dist4, Camera* c) {
    if (!K4 || !dist4) return fail(ORB_EINVAL, "camera matrix / distortion coefficients are NULL");
    if (!(K4[0] != 0.0f) || !(K4[1] != 0.0f) || !std::isfinite(K4[0]) || !std::isfinite(K4[1]))
        return fail(ORB_EINVAL, "fx and fy must be finite and non-zero");
    *c = Camera{K4[0], K4[1], K4[2], K4[3], dist4[0], dist4[1], dist4[2], dist4[3]};
    return ORB_OK;
}

// Synchronous host-buffer call through the calling thread's context: `bytes_in` staged in,
// `launch` run on the context stream with the device copy at `d`, `bytes_out` read back from
// d + out_off into `out`.
template <class F>
int host_call(int device, const void* in, size_t bytes_in, size_t out_off, size_t bytes_out, void* out, F launch) {
    if (device < 0) FCHK(hipGetDevice(&device));
    OrbHostCtx* C = orb_internal_thread_ctx(device);
    if (!C) return fail(ORB_EINVAL, "device ordinal out of range");
    const size_t total = out_off + bytes_out;
    if (int r = C->reserve(total, total)) return r;
    std::memcpy(C->pinned, in, bytes_in);
    FCHK(hipMemcpyAsync(C->buf, C->pinned, bytes_in, hipMemcpyHostToDevice, C->stream));
    launch(C->buf, C->stream);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(C->pinned + out_off, C->buf + out_off, bytes_out, hipMemcpyDeviceToHost, C->stream);
    const hipError_t es = hipStreamSynchronize(C->stream);  // the staging is reused by the next call
    if (e == hipSuccess) e = es;
    if (e != hipSuccess) return fail(ORB_EDEVICE, std::string("undistort: ") + hipGetErrorString(e));
    std::memcpy(out, C->pinned + out_off, bytes_out);
    return ORB_OK;
}

}  // namespace

extern "C" {

int orb_undistort_keypoints_batch_device(const orb_keypoint_t* d_kps, const int32_t* d_counts, int cap, int B,
                                         const float* K4, const float* dist4, orb_keypoint_t* d_kps_un,
                                         void* stream) {
    if (!d_kps || !d_counts || !d_kps_un || cap <= 0 || B < 0) return fail(ORB_EINVAL, "bad arguments");
    Camera cam;
    if (int r = camera_of(K4, dist4, &cam)) return r;
    if (B == 0) return ORB_OK;
    const long long n = (long long)B * cap;
    hipLaunchKernelGGL(k_undistort, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_kps,
                       d_counts, cap, B, cam, d_kps_un);
    FCHK(hipGetLastError());
    return ORB_OK;
}

int orb_undistort_keypoints(const orb_keypoint_t* kps, int n, const float* K4, const float* dist4, int device,
                            orb_keypoint_t* out) {
    if (n < 0 || (n && (!kps || !out))) return fail(ORB_EINVAL, "bad arguments");
    Camera cam;
    if (int r = camera_of(K4, dist4, &cam)) return r;
    if (n == 0) return ORB_OK;
    const size_t rec = sizeof(orb_keypoint_t) * (size_t)n, al = (rec + 255) & ~(size_t)255;
    // staging: [records in | counts (n) | records out]
    std::string in(al + 256, '\0');
    std::memcpy(&in[0], kps, rec);
    std::memcpy(&in[al], &n, 4);
    return host_call(device, in.data(), in.size(), al + 256, rec, out, [&](uint8_t* d, hipStream_t s) {
        hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, s, (const orb_keypoint_t*)d,
                           (const int32_t*)(d + al), n, 1, cam, (orb_keypoint_t*)(d + al + 256));
    });
}

int orb_undistort_points(const float* xy, int n, const float* K4, const float* dist4, int device, float* out) {
    if (n < 0 || (n && (!xy || !out))) return fail(ORB_EINVAL, "bad arguments");
    Camera cam;
    if (int r = camera_of(K4, dist4, &cam)) return r;
    if (n == 0) return ORB_OK;
    const size_t bytes = 8 * (size_t)n, al = (bytes + 255) & ~(size_t)255;
    return host_call(device, xy, bytes, al, bytes, out, [&](uint8_t* d, hipStream_t s) {
        hipLaunchKernelGGL(k_undistort_points, dim3((n + 255) / 256), dim3(256), 0, s, (const float*)d, n, cam,
                           (float*)(d + al));
    });
}

int orb_compute_image_bounds(int cols, int rows, const float* K4, const float* dist4, int device,
                             orb_frame_bounds_t* out) {
    if (cols <= 0 || rows <= 0 || !out) return fail(ORB_EINVAL, "bad arguments");
    Camera cam;
    if (int r = camera_of(K4, dist4, &cam)) return r;
    if (dist4[0] != 0.0f) {  // Frame.cc:323-340: the undistorted image corners
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float m[8];
        if (int r = orb_undistort_points(c, 4, K4, dist4, device, m)) return r;
        out->min_x = (int)std::fmin(std::floor(m[0]), std::floor(m[4]));
        out->max_x = (int)std::fmax(std::ceil(m[2]), std::ceil(m[6]));
        out->min_y = (int)std::fmin(std::floor(m[1]), std::floor(m[3]));
        out->max_y = (int)std::fmax(std::ceil(m[5]), std::ceil(m[7]));
    } else {  // Frame.cc:342-347
        out->min_x = 0;
        out->max_x = cols;
        out->min_y = 0;
        out->max_y = rows;
    }
    return ORB_OK;
}

}  // extern "C"
