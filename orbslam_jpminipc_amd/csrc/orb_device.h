// orb_device.h — device-side primitives of the ORB front end (gfx950).
//
// Everything here reproduces a reference-side arithmetic rule bit-for-bit; the rule and its
// source are cited per function.  Compiled with -ffp-contract=off: the only fused
// multiply-adds are the explicit __builtin_fmaf calls that mirror g++ -O3 -march=native's
// contraction of the reference (CMakeLists.txt:13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbdev {

constexpr int EDGE = 16;           // EDGE_THRESHOLD, ORBextractor.cc:77
constexpr int HALF_PATCH = 15;     // HALF_PATCH_SIZE, ORBextractor.cc:76

// cv::borderInterpolate(p, len, BORDER_REFLECT_101) (OpenCV 2.4).
__host__ __device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// cv::fastAtan2 (OpenCV 2.4 mathfuncs.cpp): float, no contraction.
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON
    // the two branches of the reference share one division: c = min / (max + eps)
    const float ax = fabsf(x), ay = fabsf(y);
    const bool ge = ax >= ay;
    const float c = (ge ? ay : ax) / ((ge ? ax : ay) + eps), c2 = c * c;
    const float poly = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    float a = ge ? poly : 90.f - poly;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// glibc 2.35 sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h) for
// |x| < 120: the reference's `(float)cos(angle)`, `(float)sin(angle)` with
// `using namespace std` resolve to cosf/sinf (ORBextractor.cc:160).  Checked bit-exact
// against glibc over every float in [0, 2*pi] (scripts/check_trig_exhaustive.c).
struct SinCosTab {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }
__device__ __forceinline__ float sincos_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2, s1 = p.s2 + x2 * p.s3, x7 = x3 * x2, s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2, c2 = p.c3 + x2 * p.c4, c1 = p.c0 + x2 * p.c1, x6 = x4 * x2, c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
}
// Returns cos in *c, sin in *s for y in [0, 120).  sinf and cosf share the reduction; each
// polynomial is evaluated once (glibc picks sin / cos polynomial by n's parity, and table
// t1 = t0 with every cos coefficient negated: the cos polynomial negates exactly).
__device__ __forceinline__ void glibc_sincosf(float y, float* s_out, float* c_out) {
    const SinCosTab t0 = {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0,
                          -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10,
                          0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
                          -0x1.994eb3774cf24p-13};
    double x = y;
    int n = 0;
    if (abstop12(y) >= abstop12(0x1.921FB6p-1f)) {  // |y| >= pi/4: x = y - n pi/2
        const double r = x * t0.hpi_inv;
        n = ((int32_t)r + 0x800000) >> 24;
        x = x - n * t0.hpi;
    }
    const double xs = ((n + 1) & 2) ? -x : x;  // x * sign[n & 3]
    const double x2 = x * x;
    const float S = sincos_poly(xs, x2, t0, 0);
    float C = sincos_poly(xs, x2, t0, 1);
    if (n & 2) C = -C;
    if (abstop12(y) < abstop12(0x1p-12f)) {
        *s_out = y;
        *c_out = 1.0f;
        return;
    }
    *s_out = (n & 1) ? C : S;
    *c_out = (n & 1) ? S : C;
}

// Minimum over each aligned group of 8 lanes (DPP: quad_perm xor 1, xor 2, row_half_mirror).
__device__ __forceinline__ uint32_t min8(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
}

// DescriptorDistance (ORBmatcher.cc:1794-1810): popcount of the 256-bit XOR.
__device__ __forceinline__ int hamming256(const uint32_t* a, const uint32_t* b) {
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d += __popc(a[i] ^ b[i]);
    return d;
}

// FAST-9/16 strength S(p) = max over the 16 arcs of 9 contiguous circle pixels of the
// minimum contrast on either side.  A pixel is a FAST corner at threshold t iff S > t, and
// its score is cornerScore<16> = S - 1 (OpenCV 2.4 fast.cpp).
// `c[16]` are the circle pixels in OpenCV's order, v the centre.  Returns 0 when S <= tmin.
__device__ __forceinline__ int fast_strength(int v, const int* c, int tmin) {
    uint32_t bright = 0, dark = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        bright |= (uint32_t)(c[k] > v + tmin) << k;
        dark |= (uint32_t)(c[k] < v - tmin) << k;
    }
    auto has9 = [](uint32_t m) {
        uint32_t m32 = m | (m << 16);
        uint32_t a = m32 & (m32 >> 1);
        uint32_t b = a & (a >> 2);
        uint32_t c4 = b & (b >> 4);
        return (c4 & (m32 >> 8) & 0xFFFFu) != 0;
    };
    if (!has9(bright) && !has9(dark)) return 0;
    int d[25];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - c[k];
#pragma unroll
    for (int k = 16; k < 25; ++k) d[k] = d[k - 16];
    int A = -1000, Bn = -1000;  // max over arcs of min(d), of min(-d)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int mn = d[k], mx = d[k];
#pragma unroll
        for (int j = 1; j < 9; ++j) {
            mn = min(mn, d[k + j]);
            mx = max(mx, d[k + j]);
        }
        A = max(A, mn);
        Bn = max(Bn, -mx);
    }
    return max(A, Bn);
}

// ---- wave64 cross-lane arithmetic on DPP (VALU only) ---------------------------------------
// __shfl_up / __shfl_xor compile to ds_bpermute_b32: every step is an LDS round trip.  DPP
// moves data between lanes inside the VALU instruction: row_shr:n within each 16-lane row,
// row_bcast:15 / row_bcast:31 across rows (GFX9 DPP16).
// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
// Sum over the 64 lanes, wave-uniform.
__device__ __forceinline__ int wave_total(int v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }
// m's bit for the calling lane ? if_set : if_clear, with the ballot mask itself as the condition
// (v_cndmask on the SGPR pair: the compiler would otherwise compare the ballot's operand again)
__device__ __forceinline__ int select_by_mask(uint64_t m, int if_clear, int if_set) {
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
    return r;
}
// Set bits of a ballot mask below the calling lane: the lane's slot in a ballot-compacted append
// (v_mbcnt_lo / v_mbcnt_hi on the mask's SGPR halves; popcount(m & lanes-below mask) took two
// v_and and two v_bcnt on a per-lane VGPR mask)
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Minimum over the 64 lanes, wave-uniform: min8 (quad_perm, row_half_mirror), row_mirror, then
// row_bcast:15 / row_bcast:31 across rows (an LDS-free butterfly; __shfl_xor pays six
// ds_bpermute round trips).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min8(v);
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xf, 0xf, false));  // row_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// The value of lane ^ 1.
__device__ __forceinline__ int lane_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false); }

}  // namespace orbdev
