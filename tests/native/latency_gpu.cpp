// Per-call latency of the reference's per-frame entry points, timed in C++ (no Python in the
// loop) the way Tracking calls them:
//   (*mpORBextractor)(im, mask, mvKeys, mDescriptors)                            Frame.cc:60
//   ORBmatcher(0.9, true).SearchForInitialization(F1, F2, prev, m12, 100)        Tracking.cc:392-393
//   ORBmatcher(0.7, true).SearchByBoW(mpReferenceKF, mCurrentFrame, matches)      Tracking.cc:927
//   ORBmatcher(0.9).SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th)      Tracking.cc:1139
// on synthetic frames 0 and 1 of stream 0 (W x H, nfeatures given).  Prints one JSON object:
// microseconds per call (median and mean over `reps` calls after warm-up) for each.
// Usage: latency_gpu W H NFEATURES REPS
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/orb_abi.h"

extern "C" int orb_synth_stream(int W, int H, uint64_t stream, uint64_t first, int count, uint8_t* out, int stride,
                                int64_t frame_stride);  // orbslam_jpminipc_amd/csrc/synth.c

namespace {

using Clock = std::chrono::steady_clock;

template <class F>
void timeit(const char* name, int reps, F&& f, bool last) {
    for (int i = 0; i < 10; ++i)
        if (f() != 0) {
            std::fprintf(stderr, "%s failed\n", name);
            std::exit(5);
        }
    std::vector<double> us(reps);
    for (int i = 0; i < reps; ++i) {
        const auto t0 = Clock::now();
        f();
        us[i] = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
    }
    double mean = 0;
    for (double u : us) mean += u;
    mean /= reps;
    std::sort(us.begin(), us.end());
    std::printf("\"%s\": {\"median_us\": %.2f, \"mean_us\": %.2f, \"p90_us\": %.2f}%s", name, us[reps / 2], mean,
                us[(reps * 9) / 10], last ? "" : ", ");
}

orb_frame_view_t view(const std::vector<orb_keypoint_t>& k, const std::vector<uint8_t>& d, int W, int H) {
    orb_frame_view_t v{};
    v.kps = k.data();
    v.desc = d.data();
    v.n = (int32_t)k.size();
    v.nlevels = 8;
    v.bounds = {0, W, 0, H};
    v.scale_factors[0] = v.level_sigma2[0] = 1.0f;  // Frame.cc:95-103
    for (int i = 1; i < 8; ++i) {
        v.scale_factors[i] = v.scale_factors[i - 1] * 1.2f;
        v.level_sigma2[i] = v.scale_factors[i] * v.scale_factors[i];
    }
    v.fx = v.fy = 500.0f;
    v.cx = W * 0.5f;
    v.cy = H * 0.5f;
    v.Rcw[0] = v.Rcw[4] = v.Rcw[8] = 1.0f;
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 5) {
        std::fprintf(stderr, "usage: latency_gpu W H NFEATURES REPS\n");
        return 2;
    }
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]), NF = std::atoi(argv[3]), reps = std::atoi(argv[4]);
    std::vector<uint8_t> frames((size_t)2 * W * H);
    if (orb_synth_stream(W, H, 0, 0, 2, frames.data(), W, (int64_t)W * H) != 0) return 3;
    orb_extractor_t* h = nullptr;
    if (orb_extractor_create(NF, 1.2f, 8, 1, 20, 0, 1, &h) != 0) return 4;
    const int cap = orb_get_max_keypoints(h);
    std::vector<orb_keypoint_t> k[2];
    std::vector<uint8_t> d[2];
    for (int f = 0; f < 2; ++f) {
        k[f].resize(cap);
        d[f].resize((size_t)cap * 32);
        int n = 0;
        if (orb_extract(h, frames.data() + (size_t)f * W * H, W, H, W, k[f].data(), cap, d[f].data(), &n) != 0)
            return 4;
        k[f].resize(n);
        d[f].resize((size_t)n * 32);
    }
    const int n1 = (int)k[0].size(), n2 = (int)k[1].size();
    std::vector<float> prev0((size_t)n1 * 2), prev((size_t)n1 * 2);
    for (int i = 0; i < n1; ++i) prev0[2 * i] = k[0][i].x, prev0[2 * i + 1] = k[0][i].y;
    std::vector<int32_t> m12(n1);
    std::vector<orb_keypoint_t> kout(cap);
    std::vector<uint8_t> dout((size_t)cap * 32);
    // BoW: one FeatureVector node per 16 keypoints in index order (the vocabulary's role is to
    // bucket; the matcher cost depends on the bucket sizes, ~10 per node at levelsup 4)
    auto fv_of = [](int n, std::vector<uint32_t>& nodes, std::vector<int32_t>& off, std::vector<int32_t>& feat) {
        for (int i = 0; i < n; ++i) {
            if (i % 16 == 0) {
                nodes.push_back((uint32_t)(i / 16));
                off.push_back(i);
            }
            feat.push_back(i);
        }
        off.push_back(n);
    };
    std::vector<uint32_t> nd1, nd2;
    std::vector<int32_t> of1, of2, ft1, ft2;
    fv_of(n1, nd1, of1, ft1);
    fv_of(n2, nd2, of2, ft2);
    const orb_feature_vector_t fv1{nd1.data(), of1.data(), ft1.data(), (int32_t)nd1.size()};
    const orb_feature_vector_t fv2{nd2.data(), of2.data(), ft2.data(), (int32_t)nd2.size()};
    const orb_frame_view_t V1 = view(k[0], d[0], W, H), V2 = view(k[1], d[1], W, H);
    std::vector<uint8_t> usable(n1, 1);
    std::vector<int32_t> fmatch(n2);
    // SearchByProjection(local map): every F1 keypoint as a map point projected where it was
    std::vector<float> px(n1), py(n1), vcos(n1, 1.0f);
    std::vector<int32_t> lvl(n1);
    for (int i = 0; i < n1; ++i) px[i] = k[0][i].x, py[i] = k[0][i].y, lvl[i] = k[0][i].octave;
    std::vector<int32_t> sbp(n2);
    // SearchByProjection(motion model), Tracking.cc:1078 (monocular th = 15): the last frame's
    // keypoints as map points at depth 5 in front of identical poses, so each projects where it
    // was detected; WindowSearch (ORBmatcher.cc:409-516) between the two frames, window 100
    const float fx = V1.fx, fy = V1.fy, cx = V1.cx, cy = V1.cy;
    std::vector<float> mpos((size_t)n1 * 3);
    for (int i = 0; i < n1; ++i) {
        const float z = 5.0f;
        mpos[3 * i] = (k[0][i].x - cx) / fx * z;
        mpos[3 * i + 1] = (k[0][i].y - cy) / fy * z;
        mpos[3 * i + 2] = z;
    }
    orb_map_points_t mp{};
    mp.pos = mpos.data();
    mp.n = n1;
    std::vector<int32_t> mot(n2), win(n2);
    std::printf("{\"width\": %d, \"height\": %d, \"nfeatures\": %d, \"n1\": %d, \"n2\": %d, \"reps\": %d, ", W, H, NF,
                n1, n2, reps);
    timeit("orb_extract", reps, [&] {
        int n = 0;
        return orb_extract(h, frames.data(), W, H, W, kout.data(), cap, dout.data(), &n);
    }, false);
    timeit("orb_search_for_initialization", reps, [&] {
        prev = prev0;
        int nm = 0;
        return orb_search_for_initialization(k[0].data(), d[0].data(), n1, k[1].data(), d[1].data(), n2,
                                             orb_frame_bounds_t{0, W, 0, H}, 0.9f, 1, 100, prev.data(), m12.data(), &nm);
    }, false);
    timeit("orb_search_by_bow_kf_f", reps, [&] {
        int nm = 0;
        return orb_search_by_bow_kf_f(&V1, usable.data(), fv1, &V2, fv2, 0.7f, 1, fmatch.data(), &nm, 0);
    }, false);
    timeit("orb_search_by_projection_local", reps, [&] {
        int nm = 0;
        return orb_search_by_projection_local(&V2, nullptr, n1, usable.data(), px.data(), py.data(), lvl.data(),
                                              vcos.data(), d[0].data(), 1.0f, 0.9f, sbp.data(), &nm, 0);
    }, false);
    timeit("orb_search_by_projection_motion", reps, [&] {
        int nm = 0;
        return orb_search_by_projection_motion(&V2, nullptr, &V1, mp, usable.data(), 15.0f, 1, mot.data(), &nm, 0);
    }, false);
    timeit("orb_window_search", reps, [&] {
        int nm = 0;
        return orb_window_search(&V1, usable.data(), &V2, 100, 0, 7, 0.9f, 1, win.data(), &nm, 0);
    }, true);
    std::printf("}\n");
    orb_extractor_destroy(h);
    return 0;
}
