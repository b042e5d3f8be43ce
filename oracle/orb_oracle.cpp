/*
 * orb_oracle.cpp — TEST INFRASTRUCTURE ONLY (parity checker; never shipped, never called
 * by the product path).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load liborb_oracle.so.
 *
 * A CPU restatement of the reference's per-frame ORB front end
 * (caomw/ORBSLAM_jpMiniPC @ /root/reference), written as a reading of:
 *   src/ORBextractor.cc:73-822   extractor (ctor, pyramid, per-cell FAST + retention,
 *                                 IC angle, blur, rBRIEF)
 *   src/ORBmatcher.cc:40-47, 155-284, 598-713, 715-850, 1748-1810   matcher core
 *   src/Frame.cc:56-128, 200-277  feature grid and window query
 * plus the un-vendored OpenCV 2.4 primitives those files call, restated per SURVEY.md
 * Appendix A.  The reference cannot be compiled here (it needs OpenCV 2.4, ROS and Boost,
 * none installed), so how each external behaviour is pinned is stated
 * next to it:
 *   - libstdc++ std::nth_element / std::partition: called directly (g++ 11's libstdc++,
 *     /usr/include/c++/11/bits/stl_algo.h:1964-1986) — this IS the pinned behaviour.
 *   - glibc 2.35 sinf/cosf: restated (oracle_sinf/oracle_cosf) and checked bit-exact
 *     against this host's libm sinf/cosf/sincosf over EVERY float in [0, 2*pi]
 *     (tests/test_oracle_primitives.py samples it; scripts/check_trig_exhaustive.c runs it all).
 *   - GCC -O3 -march=native FMA contraction (reference CMakeLists.txt:13): the rBRIEF
 *     sample offsets (ORBextractor.cc:166-167) are contracted by g++ 11 into
 *     fma(px, b, py*a) / fma(px, a, -(py*b)) (verified on the generated asm); the
 *     oracle writes those fmaf calls explicitly and is compiled -ffp-contract=off.
 *   - OpenCV 2.4 resize / copyMakeBorder / GaussianBlur / FAST / retainBest / fastAtan2 /
 *     cvRound: restated from the OpenCV 2.4 sources as known;
 *     there is no OpenCV in this container, so these are "parity unpinned" against a real
 *     OpenCV binary and pinned only by the known-answer tests of Appendix B.
 */
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../orbslam_jpminipc_amd/csrc/pattern31.inc"

namespace {

// ---- OpenCV 2.4 rounding helpers ------------------------------------------
inline int cvRound(double v) { return (int)lrint(v); }  // SSE2 cvtsd2si: round half to even
inline int cvFloor(double v) { return (int)std::floor(v); }
inline int cvCeil(double v) { return (int)std::ceil(v); }
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
inline short sat_s16(int v) { return (short)(v < SHRT_MIN ? SHRT_MIN : v > SHRT_MAX ? SHRT_MAX : v); }

const int PATCH_SIZE = 31;        // ORBextractor.cc:75
const int HALF_PATCH_SIZE = 15;   // ORBextractor.cc:76
const int EDGE_THRESHOLD = 16;    // ORBextractor.cc:77
const float HARRIS_K = 0.04f;     // ORBextractor.cc:73

struct KP {  // cv::KeyPoint
    float x, y, size, angle, response;
    int octave, class_id;
};

// ---- cv::borderInterpolate(BORDER_REFLECT_101) ------------------------------------------
inline int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p - 1 + 1;
        else
            p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// A level of the pyramid: (w+32) x (h+32) buffer, ROI at (16,16) (ORBextractor.cc:786-789).
struct Level {
    int w = 0, h = 0, pitch = 0;
    std::vector<uint8_t> buf;
    uint8_t* roi() { return buf.data() + (size_t)EDGE_THRESHOLD * pitch + EDGE_THRESHOLD; }
    const uint8_t* roi() const { return buf.data() + (size_t)EDGE_THRESHOLD * pitch + EDGE_THRESHOLD; }
    void alloc(int w_, int h_) {
        w = w_;
        h = h_;
        pitch = w + 2 * EDGE_THRESHOLD;
        buf.assign((size_t)pitch * (h + 2 * EDGE_THRESHOLD), 0);
    }
};

// copyMakeBorder(..., 16, BORDER_REFLECT_101) around the ROI, written in place (A1):
// left/right columns per row, then whole top/bottom rows copied (copyMakeBorder_8u).
void make_border(Level& L) {
    const int b = EDGE_THRESHOLD;
    for (int y = 0; y < L.h; ++y) {
        uint8_t* row = L.roi() + (size_t)y * L.pitch;
        for (int i = 0; i < b; ++i) row[i - b] = row[reflect101(i - b, L.w)];
        for (int i = 0; i < b; ++i) row[L.w + i] = row[reflect101(L.w + i, L.w)];
    }
    uint8_t* r0 = L.roi() - b;  // start of ROI row 0 including left border
    for (int i = 0; i < b; ++i) {
        int j = reflect101(i - b, L.h);
        std::memcpy(r0 + (ptrdiff_t)(i - b) * L.pitch, r0 + (ptrdiff_t)j * L.pitch, L.pitch);
    }
    for (int i = 0; i < b; ++i) {
        int j = reflect101(i + L.h, L.h);
        std::memcpy(r0 + (ptrdiff_t)(i + L.h) * L.pitch, r0 + (ptrdiff_t)j * L.pitch, L.pitch);
    }
}

// cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for 8U (A2): fixed-point coefficients
// (INTER_RESIZE_COEF_BITS = 11), HResizeLinear int rows, VResizeLinear with the SSE2 body
// (VResizeLinearVec_32s8u) for the leading columns and the scalar FixedPtCast tail.
int resize_linear_8u(const uint8_t* src, int sstep, int sw, int sh, uint8_t* dst, int dstep, int dw, int dh) {
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int iscale_x = (int)lrint(scale_x), iscale_y = (int)lrint(scale_y);
    bool is_area_fast = std::abs(scale_x - iscale_x) < DBL_EPSILON && std::abs(scale_y - iscale_y) < DBL_EPSILON;
    if (is_area_fast && iscale_x == 2 && iscale_y == 2) return ORB_ENOTSUP;  // OpenCV switches to INTER_AREA
    const int ONE = 2048;
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
    int xmin = 0, xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) {
            xmin = dx + 1;
            fx = 0, sx = 0;
        }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = sat_s16(cvRound(c0 * ONE));
        ialpha[2 * dx + 1] = sat_s16(cvRound(c1 * ONE));
    }
    (void)xmin;
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float c0 = 1.f - fy, c1 = fy;
        ibeta[2 * dy] = sat_s16(cvRound(c0 * ONE));
        ibeta[2 * dy + 1] = sat_s16(cvRound(c1 * ONE));
    }
    // columns handled by the SSE2 vertical body: 16-wide while x <= w-16, then 4-wide while x < w-4
    int xs = 0;
    while (xs <= dw - 16) xs += 16;
    while (xs < dw - 4) xs += 4;
    std::vector<int> H0(dw), H1(dw);
    auto hrow = [&](int sy, std::vector<int>& D) {
        sy = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);  // clip() in resizeGeneric_Invoker
        const uint8_t* S = src + (size_t)sy * sstep;
        int dx = 0;
        for (; dx < xmax; ++dx) {
            int sx = xofs[dx];
            D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
        }
        for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * ONE;
    };
    for (int dy = 0; dy < dh; ++dy) {
        hrow(yofs[dy], H0);
        hrow(yofs[dy] + 1, H1);
        int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst + (size_t)dy * dstep;
        for (int x = 0; x < dw; ++x) {
            int v;
            if (x < xs) {
                // _mm_packs_epi32(srai(H,4)) -> mulhi_epi16 with beta -> adds -> +2 >> 2 -> packus
                int h0 = std::max(-32768, std::min(32767, H0[x] >> 4));
                int h1 = std::max(-32768, std::min(32767, H1[x] >> 4));
                int m0 = (h0 * b0) >> 16, m1 = (h1 * b1) >> 16;
                int s = std::max(-32768, std::min(32767, m0 + m1));
                s = std::max(-32768, std::min(32767, s + 2));
                v = s >> 2;
            } else {
                v = (H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22;  // FixedPtCast<int,uchar,22>
            }
            D[x] = sat_u8(v);
        }
    }
    return ORB_OK;
}

// ---- FAST (cv::FAST(img, kps, t, nonmax=true) = FAST_t<16>, A4) --------------------------
const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

int corner_score16(const uint8_t* ptr, const int* pixel, int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[N];
    for (int k = 0; k < N; ++k) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

// FAST-9/16 with 3x3 non-max suppression on an image region (cols x rows at `step`):
// detection rows/cols [3, n-3), row-buffer non-max where anything outside is score 0,
// keypoints emitted row-major as KeyPoint(x, y, 7, -1, score).
void fast16(const uint8_t* img, int step, int cols, int rows, int threshold, std::vector<KP>& kps) {
    kps.clear();
    const int K = 8, N = 25;
    int pixel[25];
    for (int k = 0; k < 16; ++k) pixel[k] = kCircle[k][0] + kCircle[k][1] * step;
    for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; ++i) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols < 7 || rows < 7) return;
    std::vector<uint8_t> bufv((size_t)cols * 3, 0);
    std::vector<int> cpv((size_t)(cols + 1) * 3, 0);
    uint8_t* buf[3] = {bufv.data(), bufv.data() + cols, bufv.data() + 2 * cols};
    int* cpbuf[3] = {cpv.data() + 1, cpv.data() + cols + 2, cpv.data() + 2 * cols + 3};
    for (int i = 3; i < rows - 2; ++i) {
        const uint8_t* ptr = img + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        std::memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; ++j, ++ptr) {
                int v = ptr[0];
                const uint8_t* t = &tab[0] - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; ++k) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; ++k) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; ++k) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1]) {
                kps.push_back(KP{(float)j, (float)(i - 1), 7.f, -1.f, (float)score, 0, -1});
            }
        }
    }
}

// HarrisResponses (ORBextractor.cc:79-120) with g++ -O3 -march=native's contraction of the
// response expression: fma(-(k*s), s, fma(A, B, -(C*C))) * scale^4 (see DESIGN.md §FP policy).
void harris_responses(const uint8_t* img, int step, std::vector<KP>& pts, int blockSize, float harris_k) {
    int r = blockSize / 2;
    float scale = (1 << 2) * blockSize * 255.0f;
    scale = 1.0f / scale;
    float scale_sq_sq = scale * scale * scale * scale;
    for (auto& kp : pts) {
        int x0 = cvRound(kp.x - r), y0 = cvRound(kp.y - r);
        const uint8_t* ptr0 = img + (ptrdiff_t)y0 * step + x0;
        int a = 0, b = 0, c = 0;
        for (int i = 0; i < blockSize; ++i)
            for (int j = 0; j < blockSize; ++j) {
                const uint8_t* ptr = ptr0 + (ptrdiff_t)i * step + j;
                int Ix = (ptr[1] - ptr[-1]) * 2 + (ptr[-step + 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[step - 1]);
                int Iy = (ptr[step] - ptr[-step]) * 2 + (ptr[step - 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[-step + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        float fa = (float)a, fb = (float)b, fc = (float)c;
        float s = fa + fb;
        float t3 = harris_k * s;
        float u = std::fma(fa, fb, -(fc * fc));
        float rsp = std::fma(-t3, s, u);
        kp.response = rsp * scale_sq_sq;
    }
}

// KeyPointsFilter::retainBest (A5) followed by ORB-SLAM's truncation (ORBextractor.cc:683-685).
void retain_best(std::vector<KP>& kps, int n) {
    if (n >= 0 && kps.size() > (size_t)n) {
        if (n == 0) {
            kps.clear();
            return;
        }
        std::nth_element(kps.begin(), kps.begin() + n, kps.end(),
                         [](const KP& a, const KP& b) { return a.response > b.response; });
        float amb = kps[n - 1].response;
        auto new_end = std::partition(kps.begin() + n, kps.end(), [amb](const KP& k) { return k.response >= amb; });
        kps.resize(new_end - kps.begin());
    }
    if ((int)kps.size() > n) kps.resize(n);
}

// cv::fastAtan2 (A6): float polynomial, degrees, no contraction.
const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// glibc 2.35 sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h), the path
// for |x| < 120 (keypoint angles are in [0, 2*pi]).  Bit-exact vs this host's libm over
// every float in [0, 2*pi] with and without FMA (scripts/check_trig_exhaustive.c).
struct SinCosTab {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
const SinCosTab kSC[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

inline uint32_t abstop12(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return (u >> 20) & 0x7ff;
}
inline float sincos_poly(double x, double x2, const SinCosTab* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2, s1 = p->s2 + x2 * p->s3, x7 = x3 * x2, s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2, c2 = p->c3 + x2 * p->c4, c1 = p->c0 + x2 * p->c1, x6 = x4 * x2, c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
}
inline double reduce_fast(double x, const SinCosTab* p, int* np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - n * p->hpi;
}
float glibc_sinf(float y) {
    double x = y;
    const SinCosTab* p = &kSC[0];
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, x * x, p, 0);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = reduce_fast(x, p, &n);
        double s = p->sign[n & 3];
        if (n & 2) p = &kSC[1];
        return sincos_poly(x * s, x * x, p, n);
    }
    return std::sin(y);  // outside the keypoint-angle domain; not reached by the extractor
}
float glibc_cosf(float y) {
    double x = y;
    const SinCosTab* p = &kSC[0];
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x * x, p, 1);
    }
    if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = reduce_fast(x, p, &n);
        double s = p->sign[n & 3];
        if (n & 2) p = &kSC[1];
        return sincos_poly(x * s, x * x, p, n ^ 1);
    }
    return std::cos(y);
}

// IC_Angle (ORBextractor.cc:124-151) on the un-blurred level.
float ic_angle(const uint8_t* level_roi, int step, float px, float py, const std::vector<int>& umax) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = level_roi + (ptrdiff_t)cvRound(py) * step + cvRound(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// getGaussianKernel(7, 2, CV_32F) then convertTo(CV_32S, 1 << 8) (A3).
void gaussian_taps(int* k7) {
    const int n = 7;
    double sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX), sum = 0;
    float cf[7];
    for (int i = 0; i < n; ++i) {
        double x = i - (n - 1) * 0.5;
        double t = std::exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) cf[i] = (float)(cf[i] * sum);
    for (int i = 0; i < n; ++i) k7[i] = cvRound(cf[i] * 256.0f);
}

// GaussianBlur(level ROI, 7x7, sigma 2, BORDER_REFLECT_101) in place on a non-isolated ROI
// (ORBextractor.cc:760, A3).  Reads the un-blurred padding for taps outside the ROI.  Row
// pass: exact int.  Column pass: SymmColumnVec_32s8u (SSE2, float taps k/65536, cvtps
// round-half-even) for x < 4*floor(w/4); the scalar FixedPtCastEx tail (T + 2^15) >> 16.
void gaussian_blur_level(const Level& L, std::vector<uint8_t>& out) {
    int k[7];
    gaussian_taps(k);
    const int w = L.w, h = L.h, step = L.pitch;
    const uint8_t* roi = L.roi();
    std::vector<int> R((size_t)(h + 6) * w);
    for (int y = -3; y < h + 3; ++y) {
        const uint8_t* row = roi + (ptrdiff_t)y * step;
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int i = 0; i < 7; ++i) s += k[i] * row[x + i - 3];
            R[(size_t)(y + 3) * w + x] = s;
        }
    }
    float ky[4];
    for (int i = 0; i < 4; ++i) ky[i] = (float)((double)k[3 + i] * (1. / 65536));
    const int xsimd = (w / 4) * 4;
    out.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y) {
        const int* c = &R[(size_t)(y + 3) * w];
        for (int x = 0; x < w; ++x) {
            int v;
            if (x < xsimd) {
                float s0 = (float)c[x] * ky[0] + 0.0f;
                for (int j = 1; j <= 3; ++j) {
                    int pair = c[x + (ptrdiff_t)j * w] + c[x - (ptrdiff_t)j * w];
                    s0 = s0 + (float)pair * ky[j];
                }
                int iv = (int)lrintf(s0);  // _mm_cvtps_epi32, MXCSR round-to-nearest-even
                v = std::max(-32768, std::min(32767, iv));
            } else {
                int T = k[3] * c[x];
                for (int j = 1; j <= 3; ++j) T += k[3 + j] * (c[x + (ptrdiff_t)j * w] + c[x - (ptrdiff_t)j * w]);
                v = (T + (1 << 15)) >> 16;
            }
            out[(size_t)y * w + x] = sat_u8(v);
        }
    }
}

// computeOrbDescriptor (ORBextractor.cc:155-194).  Samples the blurred ROI inside the level
// and the un-blurred padding outside it.
const float factorPI = (float)(M_PI / 180.f);
void orb_descriptor(const KP& kpt, const Level& L, const std::vector<uint8_t>& blurred, uint8_t* desc) {
    float angle = kpt.angle * factorPI;
    float a = glibc_cosf(angle), b = glibc_sinf(angle);
    const int cy = cvRound(kpt.y), cx = cvRound(kpt.x);
    auto value = [&](int idx) -> int {
        float px = (float)kOrbPattern31[2 * idx], py = (float)kOrbPattern31[2 * idx + 1];
        int dy = cvRound(std::fma(px, b, py * a));
        int dx = cvRound(std::fma(px, a, -(py * b)));
        int y = cy + dy, x = cx + dx;
        if (x >= 0 && x < L.w && y >= 0 && y < L.h) return blurred[(size_t)y * L.w + x];
        return L.roi()[(ptrdiff_t)y * L.pitch + x];
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            int t0 = value(16 * i + 2 * bit), t1 = value(16 * i + 2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

int descriptor_distance(const uint8_t* a8, const uint8_t* b8) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a8 + 4 * i, 4);
        std::memcpy(&pb, b8 + 4 * i, 4);
        unsigned int v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

}  // namespace

// =========================================================================================
struct oracle_extractor {
    int nfeatures;
    double scaleFactor;  // a double member in the reference (ORBextractor.h:62)
    int nlevels, scoreType, fastTh;
    std::vector<float> mvScaleFactor, mvInvScaleFactor;
    std::vector<int> mnFeaturesPerLevel, umax;
    std::vector<Level> pyr;
    std::vector<std::vector<uint8_t>> blurred;
    std::vector<std::vector<int>> cellCounts;
    std::vector<int> cellRows, cellCols;

    // ORBextractor::ORBextractor (ORBextractor.cc:457-511)
    oracle_extractor(int nf, float sf, int nl, int st, int th)
        : nfeatures(nf), scaleFactor(sf), nlevels(nl), scoreType(st), fastTh(th) {
        mvScaleFactor.resize(nlevels);
        mvScaleFactor[0] = 1;
        for (int i = 1; i < nlevels; ++i) mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
        float invScaleFactor = (float)(1.0f / scaleFactor);
        mvInvScaleFactor.resize(nlevels);
        mvInvScaleFactor[0] = 1;
        for (int i = 1; i < nlevels; ++i) mvInvScaleFactor[i] = mvInvScaleFactor[i - 1] * invScaleFactor;
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0 / scaleFactor);
        float nDesiredFeaturesPerScale =
            nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; ++level) {
            mnFeaturesPerLevel[level] = cvRound(nDesiredFeaturesPerScale);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesiredFeaturesPerScale *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);
        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = cvFloor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
        int vmin = cvCeil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRound(std::sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    // ComputePyramid (ORBextractor.cc:781-822); the input is treated as a whole image.
    int compute_pyramid(const uint8_t* img, int W, int H, int stride) {
        pyr.assign(nlevels, Level());
        for (int level = 0; level < nlevels; ++level) {
            float scale = mvInvScaleFactor[level];
            int w = cvRound((float)W * scale), h = cvRound((float)H * scale);
            if (w <= 0 || h <= 0) return ORB_ENOTSUP;
            pyr[level].alloc(w, h);
            if (level != 0) {
                Level& P = pyr[level - 1];
                int st = resize_linear_8u(P.roi(), P.pitch, P.w, P.h, pyr[level].roi(), pyr[level].pitch, w, h);
                if (st) return st;
            } else {
                for (int y = 0; y < h; ++y) std::memcpy(pyr[0].roi() + (size_t)y * pyr[0].pitch, img + (size_t)y * stride, w);
            }
            make_border(pyr[level]);
        }
        return ORB_OK;
    }

    // ComputeKeyPoints (ORBextractor.cc:522-707)
    int compute_keypoints(std::vector<std::vector<KP>>& allKeypoints) {
        allKeypoints.assign(nlevels, {});
        cellCounts.assign(nlevels, {});
        cellRows.assign(nlevels, 0);
        cellCols.assign(nlevels, 0);
        float imageRatio = (float)pyr[0].w / pyr[0].h;
        for (int level = 0; level < nlevels; ++level) {
            const int nDesiredFeatures = mnFeaturesPerLevel[level];
            const int levelCols = (int)std::sqrt((float)nDesiredFeatures / (5 * imageRatio));
            const int levelRows = (int)(imageRatio * levelCols);
            if (levelCols <= 0 || levelRows <= 0) return ORB_ENOTSUP;  // reference divides by zero
            const int minBorderX = EDGE_THRESHOLD, minBorderY = minBorderX;
            const int maxBorderX = pyr[level].w - EDGE_THRESHOLD, maxBorderY = pyr[level].h - EDGE_THRESHOLD;
            const int W = maxBorderX - minBorderX, H = maxBorderY - minBorderY;
            const int cellW = (int)std::ceil((float)W / levelCols);
            const int cellH = (int)std::ceil((float)H / levelRows);
            const int nCells = levelRows * levelCols;
            const int nfeaturesCell = (int)std::ceil((float)nDesiredFeatures / nCells);
            std::vector<std::vector<std::vector<KP>>> cellKeyPoints(levelRows, std::vector<std::vector<KP>>(levelCols));
            std::vector<std::vector<int>> nToRetain(levelRows, std::vector<int>(levelCols));
            std::vector<std::vector<int>> nTotal(levelRows, std::vector<int>(levelCols));
            std::vector<std::vector<bool>> bNoMore(levelRows, std::vector<bool>(levelCols, false));
            std::vector<int> iniXCol(levelCols), iniYRow(levelRows);
            int nNoMore = 0, nToDistribute = 0;
            float hY = cellH + 6;
            Level& L = pyr[level];
            for (int i = 0; i < levelRows; ++i) {
                const float iniY = minBorderY + i * cellH - 3;
                iniYRow[i] = (int)iniY;
                if (i == levelRows - 1) {
                    hY = maxBorderY + 3 - iniY;
                    if (hY <= 0) continue;
                }
                float hX = cellW + 6;
                for (int j = 0; j < levelCols; ++j) {
                    float iniX;
                    if (i == 0) {
                        iniX = minBorderX + j * cellW - 3;
                        iniXCol[j] = (int)iniX;
                    } else {
                        iniX = iniXCol[j];
                    }
                    if (j == levelCols - 1) {
                        hX = maxBorderX + 3 - iniX;
                        if (hX <= 0) continue;
                    }
                    const int y0 = (int)iniY, y1 = (int)(iniY + hY), x0 = (int)iniX, x1 = (int)(iniX + hX);
                    if (y0 < 0 || x0 < 0 || y1 > L.h || x1 > L.w) return ORB_ENOTSUP;  // cv::Mat range assert
                    const uint8_t* cell = L.roi() + (ptrdiff_t)y0 * L.pitch + x0;
                    std::vector<KP>& ck = cellKeyPoints[i][j];
                    fast16(cell, L.pitch, x1 - x0, y1 - y0, fastTh, ck);
                    if (ck.size() <= 3) {
                        ck.clear();
                        fast16(cell, L.pitch, x1 - x0, y1 - y0, 7, ck);
                    }
                    if (scoreType == ORB_HARRIS_SCORE) harris_responses(cell, L.pitch, ck, 7, HARRIS_K);
                    const int nKeys = (int)ck.size();
                    nTotal[i][j] = nKeys;
                    if (nKeys > nfeaturesCell) {
                        nToRetain[i][j] = nfeaturesCell;
                        bNoMore[i][j] = false;
                    } else {
                        nToRetain[i][j] = nKeys;
                        nToDistribute += nfeaturesCell - nKeys;
                        bNoMore[i][j] = true;
                        nNoMore++;
                    }
                }
            }
            // Retain by score (quota redistribution, ORBextractor.cc:644-670)
            while (nToDistribute > 0 && nNoMore < nCells) {
                int nNewFeaturesCell = nfeaturesCell + (int)std::ceil((float)nToDistribute / (nCells - nNoMore));
                nToDistribute = 0;
                for (int i = 0; i < levelRows; ++i)
                    for (int j = 0; j < levelCols; ++j)
                        if (!bNoMore[i][j]) {
                            if (nTotal[i][j] > nNewFeaturesCell) {
                                nToRetain[i][j] = nNewFeaturesCell;
                                bNoMore[i][j] = false;
                            } else {
                                nToRetain[i][j] = nTotal[i][j];
                                nToDistribute += nNewFeaturesCell - nTotal[i][j];
                                bNoMore[i][j] = true;
                                nNoMore++;
                            }
                        }
            }
            std::vector<KP>& keypoints = allKeypoints[level];
            keypoints.reserve(nDesiredFeatures * 2);
            const int scaledPatchSize = (int)(PATCH_SIZE * mvScaleFactor[level]);
            cellRows[level] = levelRows;
            cellCols[level] = levelCols;
            for (int i = 0; i < levelRows; ++i)
                for (int j = 0; j < levelCols; ++j) {
                    cellCounts[level].push_back(nTotal[i][j]);
                    std::vector<KP>& keysCell = cellKeyPoints[i][j];
                    retain_best(keysCell, nToRetain[i][j]);
                    for (auto& k : keysCell) {
                        k.x += iniXCol[j];
                        k.y += iniYRow[i];
                        k.octave = level;
                        k.size = (float)scaledPatchSize;
                        keypoints.push_back(k);
                    }
                }
            if ((int)keypoints.size() > nDesiredFeatures) retain_best(keypoints, nDesiredFeatures);
        }
        for (int level = 0; level < nlevels; ++level)  // computeOrientation (ORBextractor.cc:705-706)
            for (auto& kp : allKeypoints[level]) kp.angle = ic_angle(pyr[level].roi(), pyr[level].pitch, kp.x, kp.y, umax);
        return ORB_OK;
    }

    // operator() (ORBextractor.cc:718-779)
    int extract(const uint8_t* img, int W, int H, int stride, orb_keypoint_t* out, int cap, uint8_t* desc, int* n_out) {
        *n_out = 0;
        if (W <= 0 || H <= 0) return ORB_OK;  // _image.empty(): outputs untouched
        if (!img || stride < W) return ORB_EINVAL;
        int st = compute_pyramid(img, W, H, stride);
        if (st) return st;
        std::vector<std::vector<KP>> allKeypoints;
        st = compute_keypoints(allKeypoints);
        if (st) return st;
        int nkeypoints = 0;
        for (auto& v : allKeypoints) nkeypoints += (int)v.size();
        if (nkeypoints > cap) return ORB_ERANGE;
        blurred.assign(nlevels, {});
        int offset = 0;
        for (int level = 0; level < nlevels; ++level) {
            std::vector<KP>& keypoints = allKeypoints[level];
            if (keypoints.empty()) continue;
            gaussian_blur_level(pyr[level], blurred[level]);
            for (size_t i = 0; i < keypoints.size(); ++i)
                orb_descriptor(keypoints[i], pyr[level], blurred[level], desc + (size_t)(offset + i) * 32);
            if (level != 0) {
                float scale = mvScaleFactor[level];
                for (auto& k : keypoints) {
                    k.x *= scale;
                    k.y *= scale;
                }
            }
            for (size_t i = 0; i < keypoints.size(); ++i) {
                const KP& k = keypoints[i];
                out[offset + i] = orb_keypoint_t{k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id};
            }
            offset += (int)keypoints.size();
        }
        *n_out = nkeypoints;
        return ORB_OK;
    }
};

// ---- Frame grid + matcher (Frame.cc:56-128, 200-277; ORBmatcher.cc) ----------------------
namespace {
const int FRAME_GRID_ROWS = 48, FRAME_GRID_COLS = 64;  // Frame.h:35-36
const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // ORBmatcher.cc:40-42

struct OFrame {
    const orb_keypoint_t* kps;
    const uint8_t* desc;
    int N;
    int mnMinX, mnMaxX, mnMinY, mnMaxY;
    float invW, invH;
    std::vector<std::vector<size_t>> grid;  // [ix * 48 + iy]

    OFrame(const orb_keypoint_t* k, const uint8_t* d, int n, orb_frame_bounds_t b)
        : kps(k), desc(d), N(n), mnMinX(b.min_x), mnMaxX(b.max_x), mnMinY(b.min_y), mnMaxY(b.max_y) {
        invW = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
        invH = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
        grid.assign(FRAME_GRID_COLS * FRAME_GRID_ROWS, {});
        for (int i = 0; i < N; ++i) {
            int px, py;
            if (pos_in_grid(kps[i], px, py)) grid[px * FRAME_GRID_ROWS + py].push_back(i);
        }
    }
    bool pos_in_grid(const orb_keypoint_t& kp, int& posX, int& posY) const {
        posX = (int)std::round((kp.x - mnMinX) * invW);
        posY = (int)std::round((kp.y - mnMinY) * invH);
        return !(posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS);
    }
    std::vector<size_t> features_in_area(float x, float y, float r, int minLevel, int maxLevel) const {
        std::vector<size_t> vIndices;
        int nMinCellX = (int)std::floor((x - mnMinX - r) * invW);
        nMinCellX = std::max(0, nMinCellX);
        if (nMinCellX >= FRAME_GRID_COLS) return vIndices;
        int nMaxCellX = (int)std::ceil((x - mnMinX + r) * invW);
        nMaxCellX = std::min(FRAME_GRID_COLS - 1, nMaxCellX);
        if (nMaxCellX < 0) return vIndices;
        int nMinCellY = (int)std::floor((y - mnMinY - r) * invH);
        nMinCellY = std::max(0, nMinCellY);
        if (nMinCellY >= FRAME_GRID_ROWS) return vIndices;
        int nMaxCellY = (int)std::ceil((y - mnMinY + r) * invH);
        nMaxCellY = std::min(FRAME_GRID_ROWS - 1, nMaxCellY);
        if (nMaxCellY < 0) return vIndices;
        bool bCheckLevels = true, bSameLevel = false;
        if (minLevel == -1 && maxLevel == -1)
            bCheckLevels = false;
        else if (minLevel == maxLevel)
            bSameLevel = true;
        for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
            for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
                const std::vector<size_t>& vCell = grid[ix * FRAME_GRID_ROWS + iy];
                for (size_t j = 0; j < vCell.size(); ++j) {
                    const orb_keypoint_t& kpUn = kps[vCell[j]];
                    if (bCheckLevels && !bSameLevel) {
                        if (kpUn.octave < minLevel || kpUn.octave > maxLevel) continue;
                    } else if (bSameLevel) {
                        if (kpUn.octave != minLevel) continue;
                    }
                    if (std::abs(kpUn.x - x) > r || std::abs(kpUn.y - y) > r) continue;
                    vIndices.push_back(vCell[j]);
                }
            }
        return vIndices;
    }
};

// ComputeThreeMaxima (ORBmatcher.cc:1748-1789)
void compute_three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; ++i) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2;
            max2 = max1;
            max1 = s;
            ind3 = ind2;
            ind2 = ind1;
            ind1 = i;
        } else if (s > max2) {
            max3 = max2;
            max2 = s;
            ind3 = ind2;
            ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

inline int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// FeatureVector merge walk (std::map iteration with lower_bound skips).
template <class F>
void feature_vector_walk(const uint32_t* n1, int nn1, const uint32_t* n2, int nn2, F&& body) {
    int a = 0, b = 0;
    while (a < nn1 && b < nn2) {
        if (n1[a] == n2[b]) {
            body(a, b);
            ++a;
            ++b;
        } else if (n1[a] < n2[b]) {
            a = (int)(std::lower_bound(n1, n1 + nn1, n2[b]) - n1);
        } else {
            b = (int)(std::lower_bound(n2, n2 + nn2, n1[a]) - n2);
        }
    }
}
}  // namespace

// =========================================================================================
extern "C" {

oracle_extractor_t* oracle_extractor_create(int nfeatures, float scale_factor, int nlevels, int score_type,
                                            int fast_th) {
    if (nfeatures <= 0 || nlevels <= 0 || !(scale_factor > 1.0f) || (score_type != 0 && score_type != 1))
        return nullptr;
    return new oracle_extractor(nfeatures, scale_factor, nlevels, score_type, fast_th);
}

void oracle_extractor_destroy(oracle_extractor_t* h) { delete h; }

int oracle_get_level_info(const oracle_extractor_t* h, int* fpl, float* sf, float* isf, int* umax16) {
    for (int l = 0; l < h->nlevels; ++l) {
        if (fpl) fpl[l] = h->mnFeaturesPerLevel[l];
        if (sf) sf[l] = h->mvScaleFactor[l];
        if (isf) isf[l] = h->mvInvScaleFactor[l];
    }
    if (umax16)
        for (int v = 0; v <= HALF_PATCH_SIZE; ++v) umax16[v] = h->umax[v];
    return ORB_OK;
}

int oracle_extract(oracle_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, orb_keypoint_t* kps, int cap,
                   uint8_t* desc, int* n_out) {
    return h->extract(img, w, hgt, stride, kps, cap, desc, n_out);
}

int oracle_level_image(const oracle_extractor_t* h, int l, uint8_t* out, int* w, int* hgt) {
    if (l < 0 || l >= (int)h->pyr.size()) return ORB_EINVAL;
    const Level& L = h->pyr[l];
    if (w) *w = L.w;
    if (hgt) *hgt = L.h;
    if (out) std::memcpy(out, L.buf.data(), L.buf.size());
    return ORB_OK;
}

int oracle_level_blurred(const oracle_extractor_t* h, int l, uint8_t* out) {
    if (l < 0 || l >= (int)h->blurred.size() || h->blurred[l].empty()) return ORB_EINVAL;
    std::memcpy(out, h->blurred[l].data(), h->blurred[l].size());
    return ORB_OK;
}

int oracle_cell_counts(const oracle_extractor_t* h, int l, int* rows, int* cols, int* counts, int cap) {
    if (l < 0 || l >= (int)h->cellCounts.size()) return ORB_EINVAL;
    *rows = h->cellRows[l];
    *cols = h->cellCols[l];
    int n = (int)h->cellCounts[l].size();
    if (n > cap) return ORB_ERANGE;
    for (int i = 0; i < n; ++i) counts[i] = h->cellCounts[l][i];
    return n;
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
float oracle_sinf(float x) { return glibc_sinf(x); }
float oracle_cosf(float x) { return glibc_cosf(x); }
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b); }

void oracle_nth_element_greater(const float* keys, int32_t* idx, int n, int nth) {
    std::vector<std::pair<float, int32_t>> v(n);
    for (int i = 0; i < n; ++i) v[i] = {keys[idx[i]], idx[i]};
    if (nth < n)
        std::nth_element(v.begin(), v.begin() + nth, v.end(),
                         [](const std::pair<float, int32_t>& a, const std::pair<float, int32_t>& b) {
                             return a.first > b.first;
                         });
    for (int i = 0; i < n; ++i) idx[i] = v[i].second;
}

void oracle_gaussian_taps(int* taps7) { gaussian_taps(taps7); }

int oracle_rot_bin(float a1, float a2) { return rot_bin(a1, a2); }

int oracle_resize(const uint8_t* src, int sstep, int sw, int sh, uint8_t* dst, int dstep, int dw, int dh) {
    return resize_linear_8u(src, sstep, sw, sh, dst, dstep, dw, dh);
}

/* GaussianBlur(7x7, sigma 2) of a (w+32) x (h+32) padded image's ROI (out: w x h). */
int oracle_blur_padded(const uint8_t* padded, int w, int hgt, uint8_t* out) {
    Level L;
    L.alloc(w, hgt);
    std::memcpy(L.buf.data(), padded, L.buf.size());
    std::vector<uint8_t> o;
    gaussian_blur_level(L, o);
    std::memcpy(out, o.data(), o.size());
    return ORB_OK;
}

/* FAST on a region (cv::FAST(img, kps, t, true)); out: n x 3 int (x, y, score). */
int oracle_fast(const uint8_t* img, int step, int cols, int rows, int threshold, int32_t* out, int cap) {
    std::vector<KP> k;
    fast16(img, step, cols, rows, threshold, k);
    if ((int)k.size() > cap) return ORB_ERANGE;
    for (size_t i = 0; i < k.size(); ++i) {
        out[3 * i] = (int)k[i].x;
        out[3 * i + 1] = (int)k[i].y;
        out[3 * i + 2] = (int)k[i].response;
    }
    return (int)k.size();
}

int oracle_features_in_area(const orb_keypoint_t* kps, int n, orb_frame_bounds_t bounds, float x, float y, float r,
                            int min_level, int max_level, int32_t* out, int cap) {
    OFrame F(kps, nullptr, n, bounds);
    std::vector<size_t> v = F.features_in_area(x, y, r, min_level, max_level);
    if ((int)v.size() > cap) return ORB_ERANGE;
    for (size_t i = 0; i < v.size(); ++i) out[i] = (int32_t)v[i];
    return (int)v.size();
}

// SearchForInitialization (ORBmatcher.cc:598-713)
int oracle_search_for_initialization(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1,
                                     const orb_keypoint_t* kps2, const uint8_t* desc2, int n2,
                                     orb_frame_bounds_t bounds, float nnratio, int check_ori, int window,
                                     float* prev_xy, int32_t* matches12, int* n_matches) {
    OFrame F1(kps1, desc1, n1, bounds), F2(kps2, desc2, n2, bounds);
    int nmatches = 0;
    for (int i = 0; i < n1; ++i) matches12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<int> vMatchedDistance(n2, INT_MAX), vnMatches21(n2, -1);
    for (int i1 = 0; i1 < n1; ++i1) {
        int level1 = kps1[i1].octave;
        if (level1 > 0) continue;
        std::vector<size_t> vIndices2 =
            F2.features_in_area(prev_xy[2 * i1], prev_xy[2 * i1 + 1], (float)window, level1, level1);
        if (vIndices2.empty()) continue;
        const uint8_t* d1 = desc1 + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            int dist = descriptor_distance(d1, desc2 + i2 * 32);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = (int)i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    matches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) rotHist[rot_bin(kps1[i1].angle, kps2[bestIdx2].angle)].push_back(i1);
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; ++i) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : rotHist[i])
                if (matches12[idx1] >= 0) {
                    matches12[idx1] = -1;
                    nmatches--;
                }
        }
    }
    for (int i1 = 0; i1 < n1; ++i1)
        if (matches12[i1] >= 0) {
            prev_xy[2 * i1] = kps2[matches12[i1]].x;
            prev_xy[2 * i1 + 1] = kps2[matches12[i1]].y;
        }
    *n_matches = nmatches;
    return ORB_OK;
}

// SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:155-284)
int oracle_search_by_bow_kf_f(const orb_keypoint_t* kf_kps, const uint8_t* kf_desc, int n_kf, const uint8_t* kf_valid,
                              const uint32_t* kf_nodes, const int32_t* kf_off, const int32_t* kf_feat, int kf_nn,
                              const orb_keypoint_t* f_kps, const uint8_t* f_desc, int n_f, const uint32_t* f_nodes,
                              const int32_t* f_off, const int32_t* f_feat, int f_nn, float nnratio, int check_ori,
                              int32_t* out_match, int* n_matches) {
    (void)n_kf;
    for (int j = 0; j < n_f; ++j) out_match[j] = -1;
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    feature_vector_walk(kf_nodes, kf_nn, f_nodes, f_nn, [&](int a, int b) {
        for (int iKF = kf_off[a]; iKF < kf_off[a + 1]; ++iKF) {
            const int realIdxKF = kf_feat[iKF];
            if (!kf_valid[realIdxKF]) continue;
            const uint8_t* dKF = kf_desc + (size_t)realIdxKF * 32;
            int bestDist1 = INT_MAX, bestIdxF = -1, bestDist2 = INT_MAX;
            for (int iF = f_off[b]; iF < f_off[b + 1]; ++iF) {
                const int realIdxF = f_feat[iF];
                if (out_match[realIdxF] >= 0) continue;
                const int dist = descriptor_distance(dKF, f_desc + (size_t)realIdxF * 32);
                if (dist < bestDist1) {
                    bestDist2 = bestDist1;
                    bestDist1 = dist;
                    bestIdxF = realIdxF;
                } else if (dist < bestDist2) {
                    bestDist2 = dist;
                }
            }
            if (bestDist1 <= TH_LOW) {
                if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                    out_match[bestIdxF] = realIdxKF;
                    if (check_ori) rotHist[rot_bin(kf_kps[realIdxKF].angle, f_kps[bestIdxF].angle)].push_back(bestIdxF);
                    nmatches++;
                }
            }
        }
    });
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; ++i) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j : rotHist[i]) {
                out_match[j] = -1;  // vpMapPointMatches[...] = NULL; nmatches-- unconditionally
                nmatches--;
            }
        }
    }
    *n_matches = nmatches;
    return ORB_OK;
}

// SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:715-850)
int oracle_search_by_bow_kf_kf(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1, const uint8_t* valid1,
                               const uint32_t* nodes1, const int32_t* off1, const int32_t* feat1, int nn1,
                               const orb_keypoint_t* kps2, const uint8_t* desc2, int n2, const uint8_t* valid2,
                               const uint32_t* nodes2, const int32_t* off2, const int32_t* feat2, int nn2,
                               float nnratio, int check_ori, int32_t* out_match, int* n_matches) {
    for (int i = 0; i < n1; ++i) out_match[i] = -1;
    std::vector<char> vbMatched2(n2, 0);
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    feature_vector_walk(nodes1, nn1, nodes2, nn2, [&](int a, int b) {
        for (int i1 = off1[a]; i1 < off1[a + 1]; ++i1) {
            const int idx1 = feat1[i1];
            if (!valid1[idx1]) continue;
            const uint8_t* d1 = desc1 + (size_t)idx1 * 32;
            int bestDist1 = INT_MAX, bestIdx2 = -1, bestDist2 = INT_MAX;
            for (int i2 = off2[b]; i2 < off2[b + 1]; ++i2) {
                const int idx2 = feat2[i2];
                if (vbMatched2[idx2] || !valid2[idx2]) continue;
                int dist = descriptor_distance(d1, desc2 + (size_t)idx2 * 32);
                if (dist < bestDist1) {
                    bestDist2 = bestDist1;
                    bestDist1 = dist;
                    bestIdx2 = idx2;
                } else if (dist < bestDist2) {
                    bestDist2 = dist;
                }
            }
            if (bestDist1 < TH_LOW) {
                if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                    out_match[idx1] = bestIdx2;
                    vbMatched2[bestIdx2] = 1;
                    if (check_ori) rotHist[rot_bin(kps1[idx1].angle, kps2[bestIdx2].angle)].push_back(idx1);
                    nmatches++;
                }
            }
        }
    });
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        compute_three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; ++i) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j : rotHist[i]) {
                out_match[j] = -1;
                nmatches--;
            }
        }
    }
    *n_matches = nmatches;
    return ORB_OK;
}

double oracle_bench(int nfeatures, float scale_factor, int nlevels, int fast_th, const uint8_t* imgs, int B, int w,
                    int hgt, int stride, int64_t pitch, int threads, int match, int64_t* total_kps,
                    int64_t* total_matches) {
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads <= 0) threads = 1;
    std::vector<orb_keypoint_t> kps((size_t)B * nfeatures);
    std::vector<uint8_t> desc((size_t)B * nfeatures * 32);
    std::vector<int> counts(B, 0), nm(std::max(B - 1, 1), 0), status(threads, 0);
    orb_frame_bounds_t bounds{0, w, 0, hgt};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t]() {
            oracle_extractor ex(nfeatures, scale_factor, nlevels, ORB_FAST_SCORE, fast_th);
            for (int k = t; k < B; k += threads) {
                int st = ex.extract(imgs + (size_t)k * pitch, w, hgt, stride, &kps[(size_t)k * nfeatures], nfeatures,
                                    &desc[(size_t)k * nfeatures * 32], &counts[k]);
                if (st) status[t] = st;
            }
        });
    for (auto& th : pool) th.join();
    pool.clear();
    if (match) {
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&, t]() {
                std::vector<float> prev(2 * (size_t)nfeatures);
                std::vector<int32_t> m12(nfeatures);
                for (int p = t; p < B - 1; p += threads) {
                    const int f1 = p, f2 = p + 1;
                    for (int i = 0; i < counts[f1]; ++i) {
                        prev[2 * i] = kps[(size_t)f1 * nfeatures + i].x;
                        prev[2 * i + 1] = kps[(size_t)f1 * nfeatures + i].y;
                    }
                    oracle_search_for_initialization(&kps[(size_t)f1 * nfeatures], &desc[(size_t)f1 * nfeatures * 32],
                                                     counts[f1], &kps[(size_t)f2 * nfeatures],
                                                     &desc[(size_t)f2 * nfeatures * 32], counts[f2], bounds, 0.9f, 1,
                                                     100, prev.data(), m12.data(), &nm[p]);
                }
            });
        for (auto& th : pool) th.join();
    }
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int s : status)
        if (s) return -1.0;
    int64_t tk = 0, tm = 0;
    for (int c : counts) tk += c;
    for (int m : nm) tm += m;
    if (total_kps) *total_kps = tk;
    if (total_matches) *total_matches = tm;
    return dt;
}

}  // extern "C"
