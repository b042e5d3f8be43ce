// Where a host SearchForInitialization call's time goes (experiment harness): medians over 200
// repetitions of (a) an empty kernel launch + stream sync, (b) a 104 KB H2D copy from pinned
// memory + sync, (c) a 12 KB D2H copy to pinned memory + sync, (d) (b) + launch + (c) + sync on
// one stream, (e) a 104 KB host memcpy (the staging of the call's inputs), and (f) the library's
// orb_search_for_initialization on two synthetic 640x480 frames (1000 keypoints each).
// Build: hipcc --offload-arch=gfx950 -O2 -o build/sfi_breakdown scripts/sfi_breakdown.cpp
//   -Lorbslam_jpminipc_amd -lorb_hip -lsynth -Wl,-rpath,'$ORIGIN/../orbslam_jpminipc_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/orb_abi.h"

extern "C" int orb_synth_stream(int W, int H, uint64_t stream, uint64_t first, int count, uint8_t* out, int stride,
                                int64_t frame_stride);

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 1;
}

using Clock = std::chrono::steady_clock;

template <class F>
static double median_us(F&& f, int reps = 200) {
    for (int i = 0; i < 20; ++i) f();
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        const auto a = Clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(Clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    const size_t inB = 104 * 1024, outB = 12 * 1024;
    uint8_t *hin = nullptr, *hout = nullptr, *din = nullptr, *dout = nullptr;
    if (hipHostMalloc((void**)&hin, inB) != hipSuccess || hipHostMalloc((void**)&hout, outB) != hipSuccess ||
        hipMalloc((void**)&din, inB) != hipSuccess || hipMalloc((void**)&dout, outB) != hipSuccess)
        return 2;
    std::vector<uint8_t> src(inB, 7);
    const double a = median_us([&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, (int*)dout);
        (void)hipStreamSynchronize(s);
    });
    const double b = median_us([&] {
        (void)hipMemcpyAsync(din, hin, inB, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
    });
    const double c = median_us([&] {
        (void)hipMemcpyAsync(hout, dout, outB, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    });
    const double d = median_us([&] {
        (void)hipMemcpyAsync(din, hin, inB, hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(256), 0, s, (int*)dout);
        (void)hipMemcpyAsync(hout, dout, outB, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    });
    const double e = median_us([&] { std::memcpy(hin, src.data(), inB); });
    // (f) the library call
    const int W = 640, H = 480, NF = 1000;
    std::vector<uint8_t> frames((size_t)2 * W * H);
    orb_synth_stream(W, H, 0, 0, 2, frames.data(), W, (int64_t)W * H);
    orb_extractor_t* h = nullptr;
    if (orb_extractor_create(NF, 1.2f, 8, 1, 20, 0, 1, &h) != 0) return 3;
    const int cap = orb_get_max_keypoints(h);
    std::vector<orb_keypoint_t> k[2];
    std::vector<uint8_t> dd[2];
    for (int f = 0; f < 2; ++f) {
        k[f].resize(cap);
        dd[f].resize((size_t)cap * 32);
        int n = 0;
        if (orb_extract(h, frames.data() + (size_t)f * W * H, W, H, W, k[f].data(), cap, dd[f].data(), &n) != 0) return 4;
        k[f].resize(n);
    }
    const int n1 = (int)k[0].size(), n2 = (int)k[1].size();
    std::vector<float> prev0((size_t)n1 * 2), prev((size_t)n1 * 2);
    for (int i = 0; i < n1; ++i) prev0[2 * i] = k[0][i].x, prev0[2 * i + 1] = k[0][i].y;
    std::vector<int32_t> m12(n1);
    const double f = median_us([&] {
        prev = prev0;
        int nm = 0;
        orb_search_for_initialization(k[0].data(), dd[0].data(), n1, k[1].data(), dd[1].data(), n2,
                                      orb_frame_bounds_t{0, W, 0, H}, 0.9f, 1, 100, prev.data(), m12.data(), &nm);
    });
    // (g) the device entry alone on resident inputs (launch + kernel + sync)
    const int cp = std::max(n1, n2);
    orb_keypoint_t* dk = nullptr;
    uint8_t* ddesc = nullptr;
    int32_t *dcnt = nullptr, *dm = nullptr;
    float* dprev = nullptr;
    if (hipMalloc((void**)&dk, (size_t)2 * cp * sizeof(orb_keypoint_t)) != hipSuccess ||
        hipMalloc((void**)&ddesc, (size_t)2 * cp * 32) != hipSuccess || hipMalloc((void**)&dcnt, 16) != hipSuccess ||
        hipMalloc((void**)&dm, (size_t)cp * 4 + 4) != hipSuccess || hipMalloc((void**)&dprev, (size_t)cp * 8) != hipSuccess)
        return 5;
    const int hc[4] = {n1, n2, 0, 1};
    (void)hipMemcpy(dk, k[0].data(), (size_t)n1 * sizeof(orb_keypoint_t), hipMemcpyHostToDevice);
    (void)hipMemcpy(dk + cp, k[1].data(), (size_t)n2 * sizeof(orb_keypoint_t), hipMemcpyHostToDevice);
    (void)hipMemcpy(ddesc, dd[0].data(), (size_t)n1 * 32, hipMemcpyHostToDevice);
    (void)hipMemcpy(ddesc + (size_t)cp * 32, dd[1].data(), (size_t)n2 * 32, hipMemcpyHostToDevice);
    (void)hipMemcpy(dcnt, hc, 16, hipMemcpyHostToDevice);
    (void)hipMemcpy(dprev, prev0.data(), (size_t)n1 * 8, hipMemcpyHostToDevice);  // matched positions drift
    const double g = median_us([&] {                                              // over the repetitions
        orb_search_for_initialization_batch_device(dk, ddesc, dcnt, cp, 1, dcnt + 2, dcnt + 3, orb_frame_bounds_t{0, W, 0, H},
                                                   0.9f, 1, 100, dprev, dm, dm + cp, s);
        (void)hipStreamSynchronize(s);
    });
    std::printf("{\"launch_sync_us\": %.2f, \"h2d_104k_sync_us\": %.2f, \"d2h_12k_sync_us\": %.2f, "
                "\"h2d_launch_d2h_sync_us\": %.2f, \"host_memcpy_104k_us\": %.2f, \"sfi_call_us\": %.2f, "
                "\"sfi_device_entry_sync_us\": %.2f}\n",
                a, b, c, d, e, f, g);
    orb_extractor_destroy(h);
    return 0;
}
