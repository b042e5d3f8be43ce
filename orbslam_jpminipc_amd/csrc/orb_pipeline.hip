// orb_pipeline.hip — the front end over a camera stream, overlapped on S HIP streams.
//
// One step of the reference's per-frame front end over B consecutive frames of one camera:
// ORBextractor::operator() on every frame (Frame::Frame, src/Frame.cc:56-128) and
// ORBmatcher::SearchForInitialization between each frame and the next (Tracking::Initialize,
// src/Tracking.cc:392-393) — the path bench.py measures.  Several kernels of the path are
// latency-bound by construction (the nth_element replays of k_select, the greedy pass of
// k_match_init), so the extraction is cut into S contiguous chunks, each extracted by its own
// extractor handle on its own stream: the chunks' kernels overlap on the device (640x480,
// B = 512, extraction alone: 2.30 ms on one stream, 2.18 on two).  All B-1 pairs are then
// matched in one batch on the caller's stream after the chunks' events (matching on the chunk
// streams, beside other chunks' extraction, was slower: 2.77 ms per step vs 2.58 serial).
// Results are those of the serial path (same kernels, same inputs, disjoint outputs).  Events
// order the whole step after earlier work on the caller's stream and before later work on it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"
#include "orb_internal.h"

namespace {

int fail(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }

#define PCHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct orb_pipeline {
    int S = 0, device = 0, maxBatch = 0, cap = 0;
    std::vector<orb_extractor_t*> ext;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> extracted;
    hipEvent_t start = nullptr;
    int32_t* d_iota = nullptr;  // 0 .. maxBatch: pair (b, b+1) = (iota[b], iota[b+1])

    void release() {
        (void)hipSetDevice(device);
        for (auto s : streams) (void)hipStreamSynchronize(s);
        for (auto e : ext) orb_extractor_destroy(e);
        for (auto e : extracted) (void)hipEventDestroy(e);
        if (start) (void)hipEventDestroy(start);
        for (auto s : streams) (void)hipStreamDestroy(s);
        (void)hipFree(d_iota);
    }
};

extern "C" {

int orb_pipeline_create(int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th, int device,
                        int max_batch, int n_streams, orb_pipeline_t** out) {
    if (!out) return fail(ORB_EINVAL, "out is NULL");
    *out = nullptr;
    if (max_batch <= 0 || n_streams <= 0 || n_streams > 64) return fail(ORB_EINVAL, "bad batch / stream count");
    auto* p = new orb_pipeline();
    p->S = std::min(n_streams, max_batch);
    p->device = device;
    p->maxBatch = max_batch;
    const int chunk = (max_batch + p->S - 1) / p->S;
    for (int c = 0; c < p->S; ++c) {
        orb_extractor_t* e = nullptr;
        int st = orb_extractor_create(nfeatures, scale_factor, nlevels, score_type, fast_th, device, chunk, &e);
        if (st) {
            p->release();
            delete p;
            return st;
        }
        p->ext.push_back(e);
    }
    p->cap = orb_get_max_keypoints(p->ext[0]);
    auto bail = [&](hipError_t e, const char* what) {
        p->release();
        delete p;
        return fail(ORB_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bail(e, "hipSetDevice");
    for (int c = 0; c < p->S; ++c) {
        hipStream_t s;
        hipEvent_t a;
        if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return bail(e, "hipStreamCreate");
        p->streams.push_back(s);
        if ((e = hipEventCreateWithFlags(&a, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
        p->extracted.push_back(a);
    }
    if ((e = hipEventCreateWithFlags(&p->start, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
    std::vector<int32_t> iota(max_batch + 1);
    std::iota(iota.begin(), iota.end(), 0);
    if ((e = hipMalloc(&p->d_iota, iota.size() * 4)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMemcpy(p->d_iota, iota.data(), iota.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return bail(e, "hipMemcpy");
    *out = p;
    return ORB_OK;
}

int orb_pipeline_destroy(orb_pipeline_t* p) {
    if (!p) return ORB_OK;
    p->release();
    delete p;
    return ORB_OK;
}

int orb_pipeline_max_keypoints(const orb_pipeline_t* p) { return p ? p->cap : ORB_EINVAL; }

int orb_pipeline_streams(const orb_pipeline_t* p) { return p ? p->S : ORB_EINVAL; }

int orb_pipeline_extract_and_match(orb_pipeline_t* p, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                                   int64_t frame_pitch, orb_keypoint_t* d_kps, uint8_t* d_desc, int32_t* d_counts,
                                   orb_frame_bounds_t bounds, float nnratio, int check_ori, int window,
                                   int32_t* d_matches12, int32_t* d_nmatches, void* stream) {
    return orb_pipeline_extract_undistort_and_match(p, B, d_imgs, w, hgt, stride, frame_pitch, nullptr, nullptr, d_kps,
                                                    nullptr, d_desc, d_counts, bounds, nnratio, check_ori, window,
                                                    d_matches12, d_nmatches, stream);
}

int orb_pipeline_extract_undistort_and_match(orb_pipeline_t* p, int B, const uint8_t* d_imgs, int w, int hgt,
                                             int stride, int64_t frame_pitch, const float* K4, const float* dist4,
                                             orb_keypoint_t* d_kps, orb_keypoint_t* d_kps_un, uint8_t* d_desc,
                                             int32_t* d_counts, orb_frame_bounds_t bounds, float nnratio,
                                             int check_ori, int window, int32_t* d_matches12, int32_t* d_nmatches,
                                             void* stream) {
    if (!p || B <= 0 || !d_imgs || !d_kps || !d_desc || !d_counts || (B > 1 && (!d_matches12 || !d_nmatches)))
        return fail(ORB_EINVAL, "bad arguments");
    const bool undistort = K4 != nullptr;
    if (undistort && (!dist4 || !d_kps_un)) return fail(ORB_EINVAL, "camera given without coefficients / mvKeysUn");
    if (B > p->maxBatch) return fail(ORB_EINVAL, "B exceeds max_batch");
    PCHK(hipSetDevice(p->device));
    const hipStream_t caller = (hipStream_t)stream;
    const int S = std::min(p->S, B), cap = p->cap;
    PCHK(hipEventRecord(p->start, caller));
    for (int c = 0; c < S; ++c) {
        const int b0 = (int)((long long)B * c / S), b1 = (int)((long long)B * (c + 1) / S), n = b1 - b0;
        const hipStream_t s = p->streams[c];
        PCHK(hipStreamWaitEvent(s, p->start, 0));
        int st = orb_extract_batch_device(p->ext[c], n, d_imgs + (long long)b0 * frame_pitch, w, hgt, stride,
                                          frame_pitch, d_kps + (long long)b0 * cap, d_desc + (long long)b0 * cap * 32,
                                          d_counts + b0, s);
        if (st) return st;
        // Frame::UndistortKeyPoints on the chunk's stream (Frame.cc:69, 289-319)
        if (undistort && (st = orb_undistort_keypoints_batch_device(d_kps + (long long)b0 * cap, d_counts + b0, cap, n,
                                                                    K4, dist4, d_kps_un + (long long)b0 * cap, s)))
            return st;
        PCHK(hipEventRecord(p->extracted[c], s));
    }
    // every pair once the chunks are extracted, on the caller's stream: a matcher work-group
    // takes most of a CU's LDS, so matching beside the extraction slowed both (measured)
    for (int c = 0; c < S; ++c) PCHK(hipStreamWaitEvent(caller, p->extracted[c], 0));
    if (B > 1) {
        int st = orb_search_for_initialization_batch_device(undistort ? d_kps_un : d_kps, d_desc, d_counts, cap, B - 1,
                                                            p->d_iota,
                                                            p->d_iota + 1, bounds, nnratio, check_ori, window,
                                                            nullptr, d_matches12, d_nmatches, caller);
        if (st) return st;
    }
    return ORB_OK;
}

int orb_pipeline_profile_enable(orb_pipeline_t* p, int enable) {
    if (!p) return fail(ORB_EINVAL, "bad handle");
    for (auto e : p->ext) {
        int st = orb_profile_enable(e, enable);
        if (st) return st;
    }
    return ORB_OK;
}

int orb_pipeline_profile_read(orb_pipeline_t* p, double* stage_ms, int64_t* stage_launches, int nstages) {
    if (!p || !stage_ms || !stage_launches) return fail(ORB_EINVAL, "bad arguments");
    std::vector<double> ms(nstages);
    std::vector<int64_t> n(nstages);
    int k = 0;
    for (int i = 0; i < nstages; ++i) stage_ms[i] = 0, stage_launches[i] = 0;
    for (auto e : p->ext) {
        k = orb_profile_read(e, ms.data(), n.data(), nstages);
        if (k < 0) return k;
        for (int i = 0; i < k; ++i) {
            stage_ms[i] += ms[i];
            stage_launches[i] += n[i];
        }
    }
    return k;
}

}  // extern "C"
