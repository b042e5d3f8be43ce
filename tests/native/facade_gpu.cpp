// GPU run of the C++ facade (include/orb_slam_gpu.hpp) the way Tracking drives it:
//   (*mpORBextractor)(im, mask, mvKeys, mDescriptors)                     Frame.cc:60
//   ORBmatcher(0.9, true).SearchForInitialization(F1, F2, prev, m12, 100) Tracking.cc:392-393
//   ORBmatcher(0.9, true).WindowSearch(F1, F2, 100, matches2)             ORBmatcher.cc:409-516
// on synthetic frames 0 and 1 of stream 0 at 320 x 240 (the golden fixtures' frames,
// tests/golden/golden.json).  Writes the raw outputs into the directory given as argv[1];
// tests/test_gpu_facade.py compares them with the golden fixtures and the oracle.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/orb_slam_gpu.hpp"

extern "C" int orb_synth_stream(int W, int H, uint64_t stream, uint64_t first, int count, uint8_t* out, int stride,
                                int64_t frame_stride);  // orbslam_jpminipc_amd/csrc/synth.c

namespace {

bool dump(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, n, f) == n;
    return std::fclose(f) == 0 && ok;
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
    v.cx = 320.0f;
    v.cy = 240.0f;
    v.Rcw[0] = v.Rcw[4] = v.Rcw[8] = 1.0f;
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: facade_gpu OUTDIR\n");
        return 2;
    }
    const std::string out = argv[1];
    const int W = 320, H = 240;
    std::vector<uint8_t> frames((size_t)2 * W * H);
    if (orb_synth_stream(W, H, 0, 0, 2, frames.data(), W, (int64_t)W * H) != 0) return 3;
    try {
        ORB_SLAM::gpu::ORBextractor ext(500, 1.2f, 8, ORB_SLAM::gpu::ORBextractor::FAST_SCORE, 20);
        if (ext.GetLevels() != 8 || ext.GetScaleFactor() != 1.2f) return 4;
        std::vector<orb_keypoint_t> k[2];
        std::vector<uint8_t> d[2];
        for (int f = 0; f < 2; ++f) {
            ext(frames.data() + (size_t)f * W * H, W, H, W, k[f], d[f]);
            if (!dump(out + "/f" + std::to_string(f) + ".kps", k[f].data(), k[f].size() * sizeof(orb_keypoint_t)) ||
                !dump(out + "/f" + std::to_string(f) + ".desc", d[f].data(), d[f].size()))
                return 5;
        }
        // an empty image leaves the outputs untouched (ORBextractor.cc:721-722)
        std::vector<orb_keypoint_t> k0 = k[0];
        ext(frames.data(), 0, 0, W, k0, d[0]);
        if (k0.size() != k[0].size()) return 6;

        ORB_SLAM::gpu::ORBmatcher m(0.9f, true);
        ORB_SLAM::gpu::FrameView F1{k[0].data(), d[0].data(), (int)k[0].size(), {0, W, 0, H}};
        ORB_SLAM::gpu::FrameView F2{k[1].data(), d[1].data(), (int)k[1].size(), {0, W, 0, H}};
        std::vector<float> prev(2 * k[0].size());  // vbPrevMatched = F1.mvKeysUn (Tracking.cc:366-368)
        for (size_t i = 0; i < k[0].size(); ++i) {
            prev[2 * i] = k[0][i].x;
            prev[2 * i + 1] = k[0][i].y;
        }
        std::vector<int> m12;
        const int n = m.SearchForInitialization(F1, F2, prev, m12, 100);
        if (!dump(out + "/sfi.m12", m12.data(), m12.size() * 4) || !dump(out + "/sfi.prev", prev.data(), prev.size() * 4) ||
            !dump(out + "/sfi.n", &n, 4))
            return 7;

        const orb_frame_view_t V1 = view(k[0], d[0], W, H), V2 = view(k[1], d[1], W, H);
        std::vector<uint8_t> usable(k[0].size());  // F1 keypoints with a MapPoint: i % 3 != 0
        for (size_t i = 0; i < usable.size(); ++i) usable[i] = i % 3 != 0;
        std::vector<int> m2;
        const int nw = m.WindowSearch(V1, usable.data(), V2, 100, m2);
        if (!dump(out + "/ws.m2", m2.data(), m2.size() * 4) || !dump(out + "/ws.n", &nw, 4)) return 8;
        std::printf("facade_gpu: %zu + %zu keypoints, %d SFI matches, %d window matches\n", k[0].size(),
                    k[1].size(), n, nw);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "facade_gpu: %s\n", e.what());
        return 1;
    }
    return 0;
}
