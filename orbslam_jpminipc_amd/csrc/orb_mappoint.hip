// orb_mappoint.hip — MapPoint descriptor maintenance on the GPU (part of liborb_hip.so).
//
// MapPoint::ComputeDistinctiveDescriptors (reference src/MapPoint.cc:185-250) for many map
// points at once: among a point's observed descriptors — its keyframes' rows, in the order of
// its std::map<KeyFrame*, size_t> observations, bad keyframes skipped (204-210) — pick the one
// with the least median Hamming distance to all of them (215-244).
//
//   k_distinctive  one wave per map point.  The usable rows are compacted into LDS in order;
//                  lane i owns row i (more than 64 rows: lanes loop), and finds its median
//                  vDists[(size_t)(0.5 (N-1))] of the sorted row by a 9-step binary search on
//                  the value (count of distances <= v), the distances recomputed from LDS with
//                  the candidate row broadcast to every lane.  The wave's minimum of
//                  (median << 16 | i) is the reference's first strict minimum (`median <
//                  BestMedian`, ascending i).
// Integer arithmetic throughout: the reference's float Distances hold integers <= 256 and
// are converted back to int (vector<int> vDists, 235), exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"
#include "orb_device.h"
#include "orb_internal.h"

namespace {

#define DD_MAX_OBS 4000  // observations per point held in LDS (36 B each)

int fail(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }

#define DCHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

__global__ void __launch_bounds__(64) k_distinctive(const int32_t* __restrict__ offsets,
                                                    const uint8_t* __restrict__ desc,
                                                    const uint8_t* __restrict__ usable, int32_t* __restrict__ bestRow,
                                                    uint8_t* __restrict__ outDesc) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_d[];  // rows x 8 dwords, then row ids
    const int m = blockIdx.x, lane = threadIdx.x;
    const int r0 = offsets[m], r1 = offsets[m + 1];
    const int cap = r1 - r0;
    int* s_rows = (int*)(s_d + (size_t)cap * 8);
    // vDescriptors: the usable observations, in order (MapPoint.cc:204-210)
    int N = 0;
    for (int c0 = 0; c0 < cap; c0 += 64) {
        const int r = r0 + c0 + lane;
        const bool ok = c0 + lane < cap && (!usable || usable[r]);
        const uint64_t msk = __ballot(ok);
        if (ok) {
            const int pos = N + orbdev::lanes_below(msk);
            s_rows[pos] = r;
            const uint4* src = (const uint4*)(desc + (size_t)r * 32);
            uint4* dst = (uint4*)(s_d + (size_t)pos * 8);
            dst[0] = src[0];
            dst[1] = src[1];
        }
        N += __popcll(msk);
    }
    __syncthreads();
    if (N == 0) {  // vDescriptors.empty(): the point keeps its descriptor (212-213)
        if (lane == 0) bestRow[m] = -1;
        return;
    }
    const int kmed = (N - 1) >> 1;  // vDists[0.5*(N-1)]: the double index truncates
    uint32_t best = 0xFFFFFFFFu;
    for (int i = lane; i < N; i += 64) {
        const uint4* ai = (const uint4*)(s_d + (size_t)i * 8);
        const uint4 a0 = ai[0], a1 = ai[1];
        int lo = 0, hi = 256;
        while (lo < hi) {  // smallest v with #{j : d(i, j) <= v} > kmed
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < N; ++j) {
                const uint4* bj = (const uint4*)(s_d + (size_t)j * 8);
                const uint4 b0 = bj[0], b1 = bj[1];
                const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                              __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
                cnt += d <= mid;
            }
            if (cnt > kmed)
                hi = mid;
            else
                lo = mid + 1;
        }
        best = min(best, ((uint32_t)lo << 16) | (uint32_t)i);
    }
    best = orbdev::wave_min_u32(best);
    const int bi = (int)(best & 0xFFFFu);
    if (lane == 0) bestRow[m] = s_rows[bi];
    if (lane < 8) ((uint32_t*)(outDesc + (size_t)m * 32))[lane] = s_d[(size_t)bi * 8 + lane];
}

}  // namespace

extern "C" {

int orb_compute_distinctive_descriptors_device(int M, const int32_t* d_offsets, const uint8_t* d_desc,
                                               const uint8_t* d_usable, int max_obs, int32_t* d_best_row,
                                               uint8_t* d_out_desc, void* stream) {
    if (M < 0 || (M > 0 && (!d_offsets || !d_desc || !d_best_row || !d_out_desc)) || max_obs < 0)
        return fail(ORB_EINVAL, "bad arguments");
    if (max_obs > DD_MAX_OBS) return fail(ORB_ENOTSUP, "more than 4000 observations of one map point");
    if (((uintptr_t)d_desc & 15) != 0 || ((uintptr_t)d_out_desc & 3) != 0)
        return fail(ORB_EINVAL, "descriptors must be 16-byte aligned");
    if (M == 0) return ORB_OK;
    const size_t lds = (size_t)std::max(max_obs, 1) * 36;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_distinctive, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_distinctive, dim3(M), dim3(64), lds, (hipStream_t)stream, d_offsets, d_desc, d_usable,
                       d_best_row, d_out_desc);
    DCHK(hipGetLastError());
    return ORB_OK;
}

int orb_compute_distinctive_descriptors(int M, const int32_t* offsets, const uint8_t* desc, const uint8_t* usable,
                                        int32_t* best_row, uint8_t* out_desc, int device) {
    if (M < 0 || (M > 0 && (!offsets || !best_row || !out_desc))) return fail(ORB_EINVAL, "bad arguments");
    if (M == 0) return ORB_OK;
    int max_obs = 0;
    if (offsets[0] != 0) return fail(ORB_EINVAL, "offsets[0] must be 0");
    for (int m = 0; m < M; ++m) {
        if (offsets[m + 1] < offsets[m]) return fail(ORB_EINVAL, "offsets must be non-decreasing");
        max_obs = std::max(max_obs, offsets[m + 1] - offsets[m]);
    }
    const int R = offsets[M];
    if (R > 0 && !desc) return fail(ORB_EINVAL, "bad arguments");
    if (max_obs > DD_MAX_OBS) return fail(ORB_ENOTSUP, "more than 4000 observations of one map point");
    int ndev = 0;
    DCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ORB_EINVAL, "device ordinal out of range");
    DCHK(hipSetDevice(device));
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t oOff = 0, oDesc = al((size_t)(M + 1) * 4), oUse = al(oDesc + (size_t)R * 32),
                 oBest = al(oUse + (size_t)R), oOut = al(oBest + (size_t)M * 4), total = al(oOut + (size_t)M * 32);
    uint8_t* buf = nullptr;
    DCHK(hipMalloc(&buf, total));
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    int r = ORB_OK;
    if (e == hipSuccess) e = hipMemcpyAsync(buf + oOff, offsets, (size_t)(M + 1) * 4, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && R) e = hipMemcpyAsync(buf + oDesc, desc, (size_t)R * 32, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && R && usable) e = hipMemcpyAsync(buf + oUse, usable, (size_t)R, hipMemcpyHostToDevice, st);
    if (e == hipSuccess)  // rows the kernel leaves untouched keep the caller's descriptor
        e = hipMemcpyAsync(buf + oOut, out_desc, (size_t)M * 32, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        r = orb_compute_distinctive_descriptors_device(M, (const int32_t*)(buf + oOff), buf + oDesc,
                                                       usable ? buf + oUse : nullptr, max_obs,
                                                       (int32_t*)(buf + oBest), buf + oOut, st);
        if (r == ORB_OK) {
            e = hipMemcpyAsync(best_row, buf + oBest, (size_t)M * 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipMemcpyAsync(out_desc, buf + oOut, (size_t)M * 32, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
    }
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(buf);
    if (r) return r;
    if (e != hipSuccess) return fail(ORB_EDEVICE, std::string("distinctive descriptors: ") + hipGetErrorString(e));
    return ORB_OK;
}

}  // extern "C"
