// TEST INFRASTRUCTURE ONLY: drives the CPU oracle under AddressSanitizer + UndefinedBehavior-
// Sanitizer (`make -C oracle sanitize`, run by tests/test_oracle_sanitizers.py).  Every entry
// point the parity tests use is exercised on the workloads they use — the extractor at each
// BASELINE configuration and the edge-case frames (flat, low texture, noise, frames smaller
// than the pyramid's borders), SearchForInitialization and WindowSearch on the pairs, the
// vocabulary transform with the FeatureVector-driven SearchByBoW, colour conversion,
// ComputeDistinctiveDescriptors and the threaded CPU baseline.  Any report aborts (the build
// uses -fno-sanitize-recover=all); exit 0 means a clean run.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "orb_oracle.h"

extern "C" int orb_synth_stream(int W, int H, uint64_t stream, uint64_t first, int count, uint8_t* out, int stride,
                                int64_t frame_pitch);
extern "C" int orb_synth_special(int kind, int W, int H, uint64_t seed, uint8_t* out, int stride);

namespace {

int g_fail = 0;

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                     \
        }                                                                 \
    } while (0)

struct Out {
    std::vector<orb_keypoint_t> k;
    std::vector<uint8_t> d;
};

Out extract(int nf, int nl, int W, int H, const uint8_t* img, int expect = 0) {
    oracle_extractor_t* h = oracle_extractor_create(nf, 1.2f, nl, 1, 20);
    CHECK(h != nullptr);
    Out o;
    const int cap = nf + 64;
    o.k.resize(cap);
    o.d.resize((size_t)cap * 32);
    int n = -1;
    const int st = oracle_extract(h, img, W, H, W, o.k.data(), cap, o.d.data(), &n);
    if (st != expect) std::printf("  extract %dx%d: status %d\n", W, H, st);
    CHECK(st == expect);
    if (st != 0) {
        oracle_extractor_destroy(h);
        return o;
    }
    CHECK(n >= 0 && n <= cap);
    o.k.resize(n > 0 ? n : 0);
    o.d.resize((size_t)o.k.size() * 32);
    // the debug views the level tests read
    std::vector<uint8_t> lev((size_t)(W + 32) * (H + 32));
    int lw = 0, lh = 0;
    CHECK(oracle_level_image(h, nl - 1, lev.data(), &lw, &lh) == 0);
    if (n > 0) CHECK(oracle_level_blurred(h, 0, lev.data()) == 0);  // kept only where level 0 has keypoints
    std::vector<int> cells(4096);
    int rows = 0, cols = 0;
    CHECK(oracle_cell_counts(h, 0, &rows, &cols, cells.data(), (int)cells.size()) >= 0);
    oracle_extractor_destroy(h);
    return o;
}

orb_frame_view_t view(const Out& o, int W, int H, int nl) {
    orb_frame_view_t v{};
    v.kps = o.k.data();
    v.desc = o.d.data();
    v.n = (int32_t)o.k.size();
    v.nlevels = nl;
    v.bounds = {0, W, 0, H};
    v.scale_factors[0] = v.level_sigma2[0] = 1.0f;
    for (int i = 1; i < nl; ++i) {
        v.scale_factors[i] = v.scale_factors[i - 1] * 1.2f;
        v.level_sigma2[i] = v.scale_factors[i] * v.scale_factors[i];
    }
    v.fx = v.fy = 500.0f;
    v.cx = W * 0.5f;
    v.cy = H * 0.5f;
    v.Rcw[0] = v.Rcw[4] = v.Rcw[8] = 1.0f;
    return v;
}

void pair_checks(int nf, int nl, int W, int H, uint64_t stream) {
    std::vector<uint8_t> f((size_t)2 * W * H);
    CHECK(orb_synth_stream(W, H, stream, 0, 2, f.data(), W, (int64_t)W * H) == 0);
    Out a = extract(nf, nl, W, H, f.data()), b = extract(nf, nl, W, H, f.data() + (size_t)W * H);
    std::vector<float> prev(2 * a.k.size());
    for (size_t i = 0; i < a.k.size(); ++i) {
        prev[2 * i] = a.k[i].x;
        prev[2 * i + 1] = a.k[i].y;
    }
    std::vector<int32_t> m12(a.k.size() + 1);
    int n = -1;
    CHECK(oracle_search_for_initialization(a.k.data(), a.d.data(), (int)a.k.size(), b.k.data(), b.d.data(),
                                           (int)b.k.size(), orb_frame_bounds_t{0, W, 0, H}, 0.9f, 1, 100,
                                           prev.data(), m12.data(), &n) == 0);
    CHECK(n >= 0);
    const orb_frame_view_t v1 = view(a, W, H, nl), v2 = view(b, W, H, nl);
    std::vector<uint8_t> usable(a.k.size() + 1, 1);
    std::vector<int32_t> m21(b.k.size() + 1);
    CHECK(oracle_window_search(&v1, usable.data(), &v2, 100, 0, 1 << 30, 0.9f, 1, m21.data(), &n) == 0);
    std::vector<int32_t> area(a.k.size() + 1);
    CHECK(oracle_features_in_area_view(&v1, 0, W * 0.5f, H * 0.5f, 50.0f, -1, -1, area.data(), (int)area.size()) >= 0);
    std::printf("  pair %dx%d nf %d: %zu/%zu keypoints\n", W, H, nf, a.k.size(), b.k.size());
}

void vocabulary_checks() {
    const int k = 6, L = 3;
    std::vector<int32_t> parent;
    std::vector<uint8_t> leaf;
    std::vector<int32_t> level{0};
    int nid = 0;
    for (int depth = 1; depth <= L; ++depth) {
        std::vector<int32_t> next;
        for (int p : level)
            for (int c = 0; c < k; ++c) {
                parent.push_back(p);
                leaf.push_back(depth == L);
                next.push_back(++nid);
            }
        level = next;
    }
    const int n = (int)parent.size();
    std::vector<uint8_t> desc((size_t)n * 32);
    std::vector<double> weight(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& x : desc) x = (uint8_t)((s = s * 6364136223846793005ull + 1442695040888963407ull) >> 56);
    for (int i = 0; i < n; ++i) weight[i] = leaf[i] ? 0.25 + (i % 7) * 0.5 : 0.0;
    oracle_vocabulary_t* v = oracle_vocabulary_create(k, L, 0, 0, n, parent.data(), leaf.data(), desc.data(),
                                                      weight.data());
    CHECK(v != nullptr);
    std::vector<uint8_t> f((size_t)2 * 320 * 240);
    CHECK(orb_synth_stream(320, 240, 9, 0, 2, f.data(), 320, 320 * 240) == 0);
    Out a = extract(500, 8, 320, 240, f.data()), b = extract(500, 8, 320, 240, f.data() + 320 * 240);
    struct FV {
        std::vector<uint32_t> nodes;
        std::vector<int32_t> off, feat;
        std::vector<uint32_t> bw;
        std::vector<double> bv;
    } fv[2];
    const Out* o[2] = {&a, &b};
    for (int i = 0; i < 2; ++i) {
        const int m = (int)o[i]->k.size();
        fv[i].nodes.resize(m + 1);
        fv[i].off.resize(m + 2);
        fv[i].feat.resize(m + 1);
        fv[i].bw.resize(m + 1);
        fv[i].bv.resize(m + 1);
        int nb = 0, nn = 0;
        CHECK(oracle_vocabulary_transform(v, o[i]->d.data(), m, 1, fv[i].bw.data(), fv[i].bv.data(), &nb,
                                          fv[i].nodes.data(), fv[i].off.data(), fv[i].feat.data(), &nn) == 0);
        fv[i].nodes.resize(nn);
        uint32_t w = 0, nd = 0;
        double wt = 0;
        if (m) CHECK(oracle_vocabulary_transform_one(v, o[i]->d.data(), 1, &w, &wt, &nd) == 0);
    }
    std::vector<uint8_t> valid1(a.k.size() + 1, 1), valid2(b.k.size() + 1, 1);
    std::vector<int32_t> out(a.k.size() + b.k.size() + 1);
    int nm = 0;
    CHECK(oracle_search_by_bow_kf_kf(a.k.data(), a.d.data(), (int)a.k.size(), valid1.data(), fv[0].nodes.data(),
                                     fv[0].off.data(), fv[0].feat.data(), (int)fv[0].nodes.size(), b.k.data(),
                                     b.d.data(), (int)b.k.size(), valid2.data(), fv[1].nodes.data(), fv[1].off.data(),
                                     fv[1].feat.data(), (int)fv[1].nodes.size(), 0.6f, 1, out.data(), &nm) == 0);
    CHECK(oracle_search_by_bow_kf_f(a.k.data(), a.d.data(), (int)a.k.size(), valid1.data(), fv[0].nodes.data(),
                                    fv[0].off.data(), fv[0].feat.data(), (int)fv[0].nodes.size(), b.k.data(),
                                    b.d.data(), (int)b.k.size(), fv[1].nodes.data(), fv[1].off.data(),
                                    fv[1].feat.data(), (int)fv[1].nodes.size(), 0.7f, 1, out.data(), &nm) == 0);
    oracle_vocabulary_destroy(v);
    std::printf("  vocabulary k=%d L=%d, bow matches %d\n", k, L, nm);
}

}  // namespace

int main() {
    // extractor at the BASELINE configurations and the edge-case frames
    const struct {
        int W, H, nf;
    } cfg[] = {{640, 480, 1000}, {640, 480, 2000}, {1241, 376, 2000}, {1280, 720, 2500}};
    for (const auto& c : cfg) pair_checks(c.nf, 8, c.W, c.H, 3);
    for (int kind = 1; kind <= 3; ++kind) {
        const int W = 160, H = 120;
        std::vector<uint8_t> img((size_t)W * H);
        CHECK(orb_synth_special(kind, W, H, (uint64_t)kind, img.data(), W) == 0);
        Out o = extract(300, 4, W, H, img.data());
        std::printf("  special %d: %zu keypoints\n", kind, o.k.size());
    }
    for (int W : {8, 33, 47, 80}) {  // levels shrinking below the 16 px FAST border and 19 px edge
        std::vector<uint8_t> f((size_t)W * W);
        CHECK(orb_synth_stream(W, W, 5, 0, 1, f.data(), W, (int64_t)W * W) == 0);
        extract(200, 8, W, W, f.data(), W < 16 ? ORB_ENOTSUP : 0);  // 8 px: no FAST cell (the reference divides by zero)
    }
    vocabulary_checks();
    {  // cvtColor 3 / 4 channels, both orders
        const int W = 37, H = 21;
        std::vector<uint8_t> src((size_t)W * H * 4), dst((size_t)W * H);
        for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 37);
        for (int cn : {3, 4})
            for (int rgb : {0, 1}) CHECK(oracle_rgb_to_gray(src.data(), W, H, W * cn, cn, rgb, dst.data()) == 0);
    }
    {  // ComputeDistinctiveDescriptors on ragged observation lists (one empty)
        const int32_t off[] = {0, 3, 3, 8};
        std::vector<uint8_t> desc(8 * 32), usable(8, 1), out(3 * 32);
        for (size_t i = 0; i < desc.size(); ++i) desc[i] = (uint8_t)(i * 13 + 1);
        usable[5] = 0;
        std::vector<int32_t> best(3);
        CHECK(oracle_compute_distinctive_descriptors(3, off, desc.data(), usable.data(), best.data(), out.data()) >= 0);
    }
    {  // primitives
        std::vector<uint8_t> src(97 * 61), dst(80 * 50);
        for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 7);
        CHECK(oracle_resize(src.data(), 97, 97, 61, dst.data(), 80, 80, 50) == 0);
        std::vector<int32_t> fk(3 * 2000);
        CHECK(oracle_fast(src.data(), 97, 97, 61, 20, fk.data(), 2000) >= 0);
        std::vector<float> keys(1001);
        std::vector<int32_t> idx(1001);
        for (int i = 0; i < 1001; ++i) {
            keys[i] = (float)((i * 7919) % 101);
            idx[i] = i;
        }
        oracle_nth_element_greater(keys.data(), idx.data(), 1001, 500);
    }
    {  // the threaded CPU baseline (bench.py's cpu_baseline leg)
        const int W = 320, H = 240, B = 6;
        std::vector<uint8_t> f((size_t)B * W * H);
        CHECK(orb_synth_stream(W, H, 2, 0, B, f.data(), W, (int64_t)W * H) == 0);
        int64_t nk = 0, nm = 0;
        CHECK(oracle_bench(500, 1.2f, 8, 20, f.data(), B, W, H, W, (int64_t)W * H, 3, 1, &nk, &nm) >= 0.0);
        CHECK(nk > 0);
    }
    std::printf("sanitize_check: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}
