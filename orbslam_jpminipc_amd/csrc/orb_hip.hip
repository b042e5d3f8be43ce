// orb_hip.hip — MI355X (gfx950) ORB front end: kernels + the C ABI of include/orb_abi.h.
//
// Pipeline for a batch of B same-size frames (all device-resident, one HIP stream):
//   k_pyr0        level 0 + reflect-101 padding          (ORBextractor.cc:814-815)
//   k_pyr_resize  level l from level l-1, fused padding   (ORBextractor.cc:800-807), l = 1..L-1
//                 (k_pyr_resize_tail: the small levels of a large batch in one launch)
//   k_fast        per level tile: FAST strength at fastTh and the per-cell 3x3 NMS; survivors
//                 appended to their cell's slots          (ORBextractor.cc:560-607)
//   k_rerun       FAST(7) re-run of cells with <= 3 survivors (609-614), spread over several
//                 workgroups per (frame, level)
//   k_select      per (frame, level): raster order per cell, quota redistribution, retainBest
//                 per cell and per level — exact libstdc++ nth_element replay (622-701)
//   k_orient_desc per keypoint (one wave): IC angle on the raw level, rBRIEF on the
//                 7x7 sigma-2 blur evaluated at the sample points, keypoint record
//                                                          (ORBextractor.cc:124-194, 705-777)
//   k_match_init  per frame pair (one wave): SearchForInitialization (ORBmatcher.cc:598-713)
//
// Reference behaviour that lives in OpenCV 2.4 / libstdc++ / glibc is restated per
// SURVEY.md Appendix A; DESIGN.md lists every arithmetic rule and where it is pinned.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <chrono>
#include <vector>

#include "../../include/orb_abi.h"
#include "../../include/orb_debug.h"
#include "nth_select.h"
#include "orb_internal.h"
#include "orb_device.h"
#include "pattern31.inc"

// Translation units: orb_ilp.hip compiles this file again (ORB_TU_ILP) for k_fast and
// k_pyr_stream alone, under the max-ILP machine scheduler; this unit then leaves those two out
// and launches them through orb_ilp.hip's launchers.  ORB_ILP_SPLIT 0 keeps both here (the
// timing builds do: their probe symbols live in this unit).
#ifdef ORB_TU_ILP
#define ORB_TU_MAIN 0
#else
#define ORB_TU_MAIN 1
#endif
#ifndef ORB_ILP_SPLIT
#define ORB_ILP_SPLIT (!KF_TIMING && !PS_TIMING)
#endif
#define ORB_ILP_HERE (ORB_TU_MAIN != ORB_ILP_SPLIT)  // k_fast / k_pyr_stream defined in this unit
#define ORB_MAX_LEVELS 16
#define ORB_MAX_CELLS_PER_LEVEL 256
#define ORB_SELECT_LDS_CAP 6144
#ifndef KF_TIMING  // 1: per-phase s_memtime sums of k_fast's waves (experiment builds only)
#define KF_TIMING 0
#endif
#ifndef KR_TIMING  // 1: per-level, per-phase s_memrealtime sums of k_rerun's cell re-runs (experiments)
#define KR_TIMING 0
#endif
#if KR_TIMING
#if ORB_TU_MAIN
__device__ unsigned long long g_krtime[ORB_MAX_LEVELS][8];
#endif
#define KR_T(i) const unsigned long long krt##i = __builtin_amdgcn_s_memrealtime()
#else
#define KR_T(i)
#endif
#ifndef KS_TIMING  // 1: per-level, per-phase s_memrealtime sums of k_select's workgroups (experiments)
#define KS_TIMING 0
#endif
#if KS_TIMING
#if ORB_TU_MAIN
__device__ unsigned long long g_kstime[ORB_MAX_LEVELS][8];
#endif
#define KS_T(i) const unsigned long long kst##i = __builtin_amdgcn_s_memrealtime()
#else
#define KS_T(i)
#endif
#if KF_TIMING
__device__ unsigned long long g_kftime[8];
#define KF_T(i) const unsigned long long kft##i = __builtin_amdgcn_s_memrealtime()
#else
#define KF_T(i)
#endif
// Only switches that keep the output exact (sizes, register targets, timing probes) exist in
// this translation unit; ablations that change the output are not part of the product source.
#if defined(KL_SKIP_FAST) || defined(KL_SKIP_QUEUE) || defined(KS_SKIP_RERUN) || defined(KS_SKIP_RETAIN) || \
    defined(KS_SKIP_LEVEL_RETAIN) || defined(KF_NOATOMIC) || defined(KM_SKIP1) || defined(KM_SKIP2) || defined(PS_EXP)
#error "wrong-output ablation switches were removed from the product source"
#endif

// ======================================================================================
// error plumbing
// ======================================================================================
#if ORB_TU_MAIN
static thread_local std::string g_last_error = "";

int orb_internal_set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

static int set_err(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }
#endif

#define HIP_TRY(expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return set_err(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));         \
    } while (0)

// ======================================================================================
// geometry (host-computed, passed to kernels by value)
// ======================================================================================
struct LevelGeom {
    int w, h, pitch, ph;    // ROI size, padded row pitch, padded rows (h + 32)
    long long base;         // byte offset of this level's frame-0 buffer in the pyramid
    long long fstride;      // bytes per frame of this level (pitch * ph)
    int rows, cols;         // cell grid (reference naming: levelRows x levelCols)
    int cell0;              // first cell of the level in the per-frame cell table
    int nDesired, nfc;      // mnFeaturesPerLevel[l], nfeaturesCell
    int kpBase;             // offset of the level's slot in the per-frame keypoint list
    int xsimd_blur;         // 4 * floor(w / 4): GaussianBlur SSE2 columns
    int xs_resize, xmax;    // VResizeLinear SSE2 columns, HResizeLinear xmax (l >= 1)
    int rtab;               // offset of this level's resize table (int32 units), l >= 1
    int rtile;              // offset of this level's resize tile table (4 ints per tile), l >= 1
    int rtileS;             // the same for the short tiles of small batches (RZ_THS rows)
    float scale;            // mvScaleFactor[l]
    float size;             // (int)(31 * mvScaleFactor[l])
    int cellW, cellH;       // detection-area size of the (non-last) cells: corner -> cell bucket
    int cellWm, cellHm;     // ceil(2^32 / cellW), ceil(2^32 / cellH): n / cell = umulhi(n, m), n < 4096
    int candBase, capMax;   // cell c of the level owns candidate slots candBase + c * capMax (capMax = the
                            // level's largest NMS-survivor bound), so k_fast needs no cell table
    int detX1, detY1;       // FAST detection region [16, detX1) x [16, detY1): union of the cells' areas
    int ringX1, ringY1;     // rBRIEF samples (reach 18) of detection-region keypoints stay in
                            // [-3, ringX1) x [-3, ringY1), inside the 16-px padding
};

struct Geom {
    int L;
    int nCells;        // cells per frame (all levels)
    int candPerFrame;  // candidate slots per frame (u32)
    int kpCap;         // keypoint slots per frame (sum of nDesired)
    int selCap;        // k_select: survivors per level held in LDS (select_cap)
    int fastTh;        // clamped to [0, 255]
    int scoreType;
    int taps[4];       // Gaussian 7-tap fixed-point kernel, centre first: 55, 49, 34, 18
    int umax[16];
    unsigned long long umaxNib;  // umax[0..15] as 4-bit nibbles (k_orient_desc's disc mask)
    uint32_t odDivMagic;          // k_orient_desc: ceil(2^32 / slot groups per frame) (exact division)
    int fastCl;                   // k_fast: per-wave corner-list capacity used (FT_CL; smaller only via
                                  // orb_debug_set_fast_corner_list, to exercise the plane-scan fallback)
    LevelGeom lv[ORB_MAX_LEVELS];
};

struct CellGeom {
    int level;
    int x0, y0, hx, hy;  // ROI in level coordinates (reference iniX, iniY, hX, hY)
    int cap;             // max NMS survivors: ceil(dw/2) * ceil(dh/2)
    int candOff;         // offset in the frame's candidate area
    int skipped;         // reference `continue` on hX/hY <= 0 (nTotal stays 0, bNoMore false)
    int cornerOff;       // bucket of this cell's FAST corners in the frame's corner area (dw*dh slots)
};

// ======================================================================================
// kernels
// ======================================================================================
using namespace orbdev;

// (m & a) | (~m & b) in one VALU
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

#if ORB_TU_MAIN  // (none of them is read by k_fast / k_pyr_stream)
// bit_pattern_31_ (ORBextractor.cc:197-455) as floats, pair-major: c_patternf[2 (64 q + l) + {0, 1}]
// = (x, y) of point 8 l + q, i.e. lane l's eight points are one float2 in each of eight 512-B
// rows (k_orient_desc loads each row with one fully coalesced global_load_dwordx2, §6.1)
__constant__ float c_patternf[1024];
// IC_Angle (ORBextractor.cc:124-151 with umax, 495-510) over the 31 x 9 patch dwords n = 9 r + c
// (five 64-lane steps, n < 320; n >= 279 carry zero coefficients): c_icoff[n] = the dword's byte
// offset in k_orient_desc's window from the patch's first dword; per byte alignment sh of the
// patch in its dword row, c_ic10 / c_ic01[320 sh + n] = the signed byte coefficients u = 4c + i -
// sh - 15 / v = r - 15 of byte i where it lies inside the disc (|u| <= umax[|v|]), else 0
__constant__ uint32_t c_icoff[320];
__constant__ uint32_t c_ic10[4 * 320];
__constant__ uint32_t c_ic01[4 * 320];
// k_orient_desc's row-pass B fragments: [N-tile t][lane l] = bytes j of B[16(l >> 4) + j][16t + (l & 15)]
__constant__ uint4 c_rowB[4 * 64];  // 279 patch dwords per alignment, zero-padded to 5 x 64
// OD_SB (the shared-blur variant): the column pass's A fragments (f16), [variant v][lane l] =
// halves j of A[l & 15][k(l >> 4, j)]: out row o = l & 15 of a 16-row block, K slot (h, j) = the
// row-pass sum of input row 4h + (j & 3) of an M-tile, its low (j < 4) or high (j >= 4) byte;
// weight tap[d] (x 256 for the high byte), d = delta + 4h + (j & 3) - o, delta = the M-tile's
// first row minus the block's (v 0: 0, v 1: 16, v 2: 12 without the tile's rows 0 .. 3)
__constant__ uint4 c_colA[3 * 64];
#endif
// ---- pyramid --------------------------------------------------------------------------
// Level 0: copyMakeBorder(image, 16, BORDER_REFLECT_101); one thread per 16-byte chunk of a
// padded row (pitch is a multiple of 16).  Interior chunks (source columns [x-16, x) inside the
// row) are one 16-, four 4- or sixteen 1-byte loads depending on the source alignment and one
// 16-byte store; the two border chunks per side reflect byte by byte.
#if ORB_TU_MAIN
__global__ void __launch_bounds__(256) k_pyr0(const uint8_t* __restrict__ imgs, int stride, long long fpitch,
                                              uint8_t* __restrict__ pyr, Geom g) {
    const LevelGeom& lg = g.lv[0];
    const int nchunk = lg.pitch >> 4;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int py = i / nchunk, x16 = (i - py * nchunk) << 4;
    if (py >= lg.ph) return;
    const int b = blockIdx.y;
    const uint8_t* src = imgs + (long long)b * fpitch + (long long)reflect101(py - EDGE, lg.h) * stride;
    uint4 out;
    if (x16 >= EDGE && x16 <= lg.w) {
        const uint8_t* p = src + (x16 - EDGE);
        const uintptr_t a = (uintptr_t)p;
        if ((a & 15u) == 0) {
            out = *(const uint4*)p;
        } else if ((a & 3u) == 0) {
            const uint32_t* q = (const uint32_t*)p;
            out = make_uint4(q[0], q[1], q[2], q[3]);
        } else {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                w[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
                       ((uint32_t)p[4 * k + 3] << 24);
            out = make_uint4(w[0], w[1], w[2], w[3]);
        }
    } else {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t word = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = x16 + 4 * k + j;
                uint32_t v = 0;
                if (px < lg.w + 2 * EDGE) v = src[reflect101(px - EDGE, lg.w)];
                word |= v << (8 * j);
            }
            w[k] = word;
        }
        out = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *(uint4*)(pyr + lg.base + (long long)b * lg.fstride + (long long)py * lg.pitch + x16) = out;
}
#endif  // ORB_TU_MAIN

// Level 0 from 3- or 4-channel frames: Tracking::GrabImage's cvtColor(.., CV_RGB2GRAY /
// CV_BGR2GRAY) (Tracking.cc:202-207) fused with the padding.  OpenCV 2.4's RGB2Gray<uchar> is an
// exact fixed-point sum, (c0*p[0] + 9617*p[1] + c2*p[2] + 2^13) >> 14 with R2Y = 4899,
// G2Y = 9617, B2Y = 1868 (yuv_shift 14): (c0, c2) = (R2Y, B2Y) for RGB order, (B2Y, R2Y) for BGR.
#if ORB_TU_MAIN
__global__ void __launch_bounds__(256) k_pyr0_color(const uint8_t* __restrict__ imgs, int stride, long long fpitch,
                                                    int cn, int c0, int c2, uint8_t* __restrict__ pyr, Geom g) {
    const LevelGeom& lg = g.lv[0];
    const int b = blockIdx.z, py = blockIdx.y * 4 + threadIdx.y;
    const int x4 = (blockIdx.x * 64 + threadIdx.x) * 4;
    if (x4 >= lg.pitch || py >= lg.ph) return;
    const uint8_t* src = imgs + (long long)b * fpitch + (long long)reflect101(py - EDGE, lg.h) * stride;
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int px = x4 + i;
        uint32_t v = 0;
        if (px < lg.w + 2 * EDGE) {
            const uint8_t* p = src + (long long)reflect101(px - EDGE, lg.w) * cn;
            v = (uint32_t)((c0 * p[0] + 9617 * p[1] + c2 * p[2] + (1 << 13)) >> 14);
        }
        word |= v << (8 * i);
    }
    *(uint32_t*)(pyr + lg.base + (long long)b * lg.fstride + (long long)py * lg.pitch + x4) = word;
}
#endif  // ORB_TU_MAIN

// Stage `rows` x `units` 16-byte units (global row pitch gsu units, LDS row pitch the same
// `units`) with 256 threads, up to RZ_SB units per thread all in flight before any LDS write:
// a k_pyr_resize source tile is one memory round trip.
#define RZ_SB 8
__device__ __forceinline__ void stage_tile16(uint4* __restrict__ dst, const uint4* __restrict__ src, long long gsu,
                                             int rows, int units, int tid) {
    const int total = rows * units;
    const int dr = 256 / units, dc = 256 - dr * units;
    for (int base = 0; base < total; base += RZ_SB * 256) {
        const int i0 = base + tid;
        const int r0 = i0 / units, c0 = i0 - r0 * units;
        // every slot is loaded (past-the-end slots re-read unit 0): a conditionally assigned
        // uint4 array was placed in scratch, one private-memory round trip per tile
        uint4 v[RZ_SB];
        int r = r0, c = c0;
#pragma unroll
        for (int k = 0; k < RZ_SB; ++k) {
            const bool ok = i0 + k * 256 < total;
            v[k] = src[ok ? (long long)r * gsu + c : 0ll];
            r += dr;
            c += dc;
            if (c >= units) {
                c -= units;
                ++r;
            }
        }
#pragma unroll
        for (int k = 0; k < RZ_SB; ++k)
            if (i0 + k * 256 < total) dst[i0 + k * 256] = v[k];
    }
}


// Level l >= 1: cv::resize(level l-1, (w_l, h_l), INTER_LINEAR) for 8U:
// fixed-point HResizeLinear rows; vertical SSE2 body (VResizeLinearVec_32s8u) for x < xs,
// scalar FixedPtCast<int,uchar,22> tail; then copyMakeBorder(REFLECT_101 | ISOLATED), fused
// by evaluating the resize at the reflected coordinate of every padded pixel.
// One workgroup per RZ_TW x RZ_TH tile of the padded level: the source rectangle the tile
// reads (host table: first 16-byte column, 16-byte units, first row, rows) is staged into LDS
// in one round trip of 16-byte loads; a thread owns 4 padded columns (taps in registers) and walks the
// RZ_TH / 4 rows of its wave.  As in OpenCV, a source row's horizontal sums are computed once
// and kept (two rows in registers) while consecutive output rows reuse them.
// Every coefficient is in [0, 2050] with a0 + a1, b0 + b1 <= 2050 (checked on the host), so
// no intermediate of the reference's saturating chain can saturate: H <= 255 * 2050 = 522750,
// (H >> 4) * b < 2^27, the SSE2 sum <= 1023 and the scalar sum < 2^31; both end in [0, 255].
// The SSE2 path's (h * b) >> 16 is then mulhi(h, b << 16).
#define RZ_TW 256  // 64 lanes x 4 columns
#ifndef RZ_TH
#define RZ_TH 32
#endif
#ifndef RZ_THS
#define RZ_THS 4  // tile rows for batches below KR_SHORT_BATCH (B=1 640x480: 0.074 -> 0.035 ms for levels 1-7)
#endif
#ifndef KR_SHORT_BATCH
#define KR_SHORT_BATCH 8
#endif
// The two levels arrive by value: a Geom indexed by the runtime level was copied to scratch
// (144 B per lane of private-memory traffic per thread).
#if ORB_TU_MAIN
template <int TH>
__global__ void __launch_bounds__(256) k_pyr_resize(uint8_t* __restrict__ pyr, const int* __restrict__ rtab,
                                                    const LevelGeom lg, const LevelGeom ls) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_src[];
    const int b = blockIdx.z, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int* tt = rtab + (TH == RZ_TH ? lg.rtile : lg.rtileS) + 4 * (blockIdx.y * gridDim.x + blockIdx.x);
    const int colStart = tt[0], words = tt[1], rowMin = tt[2], nrows = tt[3];
    const uint8_t* S = pyr + ls.base + (long long)b * ls.fstride + (long long)EDGE * ls.pitch + EDGE;
    stage_tile16((uint4*)s_src, (const uint4*)(S + (long long)rowMin * ls.pitch + colStart), ls.pitch >> 4, nrows,
                 words, tid);
    const int* xofs = rtab + lg.rtab;
    const int* alpha = xofs + lg.w;
    const int* yofs = alpha + lg.w;
    const int* beta = yofs + lg.h;
    // the wave's TH / 4 row coefficients, one row per lane, fetched while the tile loads
    // (read back with readlane: no dependent global load inside the row walk)
    const int pyA = blockIdx.y * TH + wave * (TH / 4);
    const int pyB = min(pyA + TH / 4, lg.ph);
    int rowSy = 0, rowBeta = 0;
    if (lane < TH / 4 && pyA + lane < pyB) {
        const int ly = reflect101(pyA + lane - EDGE, lg.h);
        rowSy = yofs[ly];
        rowBeta = beta[ly];
    }
    const int x4 = blockIdx.x * RZ_TW + 4 * lane;
    uint32_t o0[4], o1[4], a0[4], a1[4];
    uint32_t liveMask = 0;
    bool allSimd = true;
    uint32_t simdBytes = 0;  // 0xFF in the byte of every SSE2 column
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int px = x4 + i;
        if (px < lg.w + 2 * EDGE) liveMask |= 0xFFu << (8 * i);
        const int lx = reflect101(min(px, lg.w + 2 * EDGE - 1) - EDGE, lg.w);
        const int sx = xofs[lx];
        if (lx < lg.xmax) {
            const int aa = alpha[lx];
            a0[i] = (uint32_t)(aa & 0xFFFF);
            a1[i] = (uint32_t)(aa >> 16) & 0xFFFFu;
        } else {  // HResizeLinear tail: S[sx] * ONE (sx + 1 may be past the row: not read)
            a0[i] = 2048;
            a1[i] = 0;
        }
        o0[i] = (uint32_t)(sx - colStart);
        o1[i] = (uint32_t)((a1[i] ? sx + 1 : sx) - colStart);
        allSimd = allSimd && lx < lg.xs_resize;
        if (lx < lg.xs_resize) simdBytes |= 0xFFu << (8 * i);
    }
    __syncthreads();
    if (x4 >= lg.pitch) return;
    // a wave holding a scalar-tail column computes both formulas for all its lanes and selects per
    // byte (wave-uniform: no divergent path per row); the other waves the SSE2 one alone
    const bool waveTail = __ballot(!allSimd) != 0ull;
    const bool shift4 = allSimd && !waveTail;
    const uint8_t* L = (const uint8_t*)s_src;
    const int LP = words * 16;
    // horizontal sums of source row r: H >> 4 on the SSE2 columns, H on the scalar tail
    auto hrow = [&](int r, uint32_t* h) {
        const uint8_t* R = L + (r - rowMin) * LP;
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = (uint32_t)R[o0[i]] * a0[i] + (uint32_t)R[o1[i]] * a1[i];
        if (shift4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) h[i] >>= 4;
        }
    };
    uint8_t* D = pyr + lg.base + (long long)b * lg.fstride + x4;
    // one output row from the horizontal sums hA (source row s0) and hB (s1)
    auto vrow = [&](const int py, const uint32_t bb, const uint32_t* hA, const uint32_t* hB) {
        const uint32_t b0 = bb & 0xFFFFu, b1 = bb >> 16;
        uint32_t word;
        if (!waveTail) {
            const uint32_t B0 = b0 << 16, B1 = b1 << 16;
            uint32_t r[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = (__umulhi(hA[i], B0) + __umulhi(hB[i], B1) + 2u) >> 2;
            word = r[0] | (r[1] << 8) | (r[2] << 16) | (r[3] << 24);
        } else {  // hA / hB are full sums in this wave
            uint32_t ws = 0, wc = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ws |= ((__umulhi(hA[i] >> 4, b0 << 16) + __umulhi(hB[i] >> 4, b1 << 16) + 2u) >> 2) << (8 * i);
                wc |= ((hA[i] * b0 + hB[i] * b1 + (1u << 21)) >> 22) << (8 * i);
            }
            word = bfi(simdBytes, ws, wc);
        }
        *(uint32_t*)(D + (long long)py * lg.pitch) = word & liveMask;
    };
    // rows in pairs with the source register sets in alternating roles (k_pyr_stream's
    // build_quad): a downscale row's second source row is the next row's first, already in the
    // set that row reads first, so no sums are copied between sets (tP / tQ: rows held)
    int tP = -1, tQ = -1;
    uint32_t hP[4] = {0, 0, 0, 0}, hQ[4] = {0, 0, 0, 0};
    auto src_rows = [&](const int py, int& s0, int& s1, uint32_t& bb) {
        const int sy = __builtin_amdgcn_readlane(rowSy, py - pyA);
        bb = (uint32_t)__builtin_amdgcn_readlane(rowBeta, py - pyA);
        s0 = min(max(sy, 0), ls.h - 1);
        s1 = min(max(sy + 1, 0), ls.h - 1);
    };
    for (int py = pyA; py < pyB; py += 2) {
        {
            int s0, s1;
            uint32_t bb;
            src_rows(py, s0, s1, bb);
            if (tP != s0) hrow(s0, hP), tP = s0;
            if (tQ != s1) hrow(s1, hQ), tQ = s1;
            vrow(py, bb, hP, hQ);
        }
        if (py + 1 < pyB) {
            int s0, s1;
            uint32_t bb;
            src_rows(py + 1, s0, s1, bb);
            if (tQ != s0) hrow(s0, hQ), tQ = s0;
            if (tP != s1) hrow(s1, hP), tP = s1;
            vrow(py + 1, bb, hQ, hP);
        }
    }
}
#endif  // ORB_TU_MAIN

// Levels lf .. L-1 of one frame per 1024-thread workgroup (the small levels: one launch
// instead of one per level, each of which was latency-bound at a few thousand pixels per
// frame).  Level lf reads level lf-1 from HBM; every later level reads its source ROI from
// LDS, where the previous level left it (ping-pong buffers A / B); the level's resize tables
// are staged in LDS too.  Per padded pixel the arithmetic is k_pyr_resize's: HResizeLinear
// taps (tail columns S[sx] * 2048), then the SSE2 vertical body (((H >> 4) * b) >> 16 summed,
// + 2 >> 2) on columns lx < xs, the scalar FixedPtCast (+ 2^21 >> 22) on the others.
#define RT_THREADS 1024
#define RT_LDS_MAX (150 * 1024)
#ifndef KR_TAIL  // 0: every level by k_pyr_resize (experiment switch)
#define KR_TAIL 1
#endif
#if ORB_TU_MAIN
__global__ void __launch_bounds__(RT_THREADS) k_pyr_resize_tail(uint8_t* __restrict__ pyr,
                                                                const int* __restrict__ rtab, Geom g, int lf,
                                                                int bufA, int bufB) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_rt[];
    const int b = blockIdx.x, tid = threadIdx.x;
    int* tab = (int*)(s_rt + bufA + bufB);
    for (int l = lf; l < g.L; ++l) {
        const LevelGeom lg = g.lv[l], ls = g.lv[l - 1];
        const int w = lg.w, h = lg.h, sw = ls.w, sh = ls.h;
        const int* src = rtab + lg.rtab;
        for (int i = tid; i < 2 * (w + h); i += RT_THREADS) tab[i] = src[i];
        __syncthreads();
        const int *xofs = tab, *alpha = tab + w, *yofs = tab + 2 * w, *beta = yofs + h;
        const uint8_t* Sg = pyr + ls.base + (long long)b * ls.fstride + (long long)EDGE * ls.pitch + EDGE;
        // level l-lf even -> buffer A at 0, odd -> buffer B at bufA (bufB: B's size)
        const uint8_t* Sl = s_rt + (((l - 1 - lf) & 1) ? bufA : 0);  // level l-1's ROI (l > lf)
        uint8_t* Dl = (l + 1 < g.L) ? s_rt + (((l - lf) & 1) ? bufA : 0) : nullptr;
        const long long spitch = l > lf ? sw : ls.pitch;
        const uint8_t* S = l > lf ? Sl : Sg;
        uint8_t* D = pyr + lg.base + (long long)b * lg.fstride;
        const int nw = lg.pitch >> 2, rowsPerPass = RT_THREADS / nw;
        const int r0 = tid / nw, c4 = (tid - r0 * nw) * 4;
        if (r0 < rowsPerPass) {
            int sx[4], sx1[4];
            uint32_t a0[4], a1[4];
            bool simd[4], live[4], roiX[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = c4 + j;
                live[j] = px < w + 2 * EDGE;
                roiX[j] = px >= EDGE && px < EDGE + w;
                const int lx = reflect101(min(px, w + 2 * EDGE - 1) - EDGE, w);
                sx[j] = xofs[lx];
                if (lx < lg.xmax) {
                    const int aa = alpha[lx];
                    a0[j] = (uint32_t)(aa & 0xFFFF);
                    a1[j] = (uint32_t)(aa >> 16) & 0xFFFFu;
                } else {
                    a0[j] = 2048;
                    a1[j] = 0;
                }
                sx1[j] = a1[j] ? sx[j] + 1 : sx[j];
                simd[j] = lx < lg.xs_resize;
            }
            // four rows per step, all their source bytes loaded before any is used: the first
            // fused level reads HBM / L2, and a thread's rows would otherwise be one exposed
            // round trip each
            for (int py0 = r0; py0 < lg.ph; py0 += 4 * rowsPerPass) {
                uint32_t v[4][4][4];
                uint32_t bk[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int py = min(py0 + k * rowsPerPass, lg.ph - 1);
                    const int ly = reflect101(py - EDGE, h);
                    const int sy = yofs[ly];
                    bk[k] = (uint32_t)beta[ly];
                    const uint8_t* R0 = S + min(max(sy, 0), sh - 1) * spitch;
                    const uint8_t* R1 = S + min(max(sy + 1, 0), sh - 1) * spitch;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v[k][j][0] = R0[sx[j]];
                        v[k][j][1] = R0[sx1[j]];
                        v[k][j][2] = R1[sx[j]];
                        v[k][j][3] = R1[sx1[j]];
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int py = py0 + k * rowsPerPass;
                    if (py >= lg.ph) break;
                    const uint32_t b0 = bk[k] & 0xFFFFu, b1 = bk[k] >> 16;
                    const bool roiY = Dl && py >= EDGE && py < EDGE + h;
                    uint32_t word = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t hA = v[k][j][0] * a0[j] + v[k][j][1] * a1[j];
                        const uint32_t hB = v[k][j][2] * a0[j] + v[k][j][3] * a1[j];
                        const uint32_t r = simd[j]
                                               ? (__umulhi(hA >> 4, b0 << 16) + __umulhi(hB >> 4, b1 << 16) + 2u) >> 2
                                               : (hA * b0 + hB * b1 + (1u << 21)) >> 22;
                        if (live[j]) word |= r << (8 * j);
                        if (roiY && roiX[j]) Dl[(py - EDGE) * w + (c4 + j - EDGE)] = (uint8_t)r;
                    }
                    *(uint32_t*)(D + (long long)py * lg.pitch + c4) = word;
                }
            }
        }
        __syncthreads();  // level l complete in LDS; the tables are free
    }
}
#endif  // ORB_TU_MAIN

// ---- the whole pyramid of a frame in one streaming pass (large batches) ------------------
// k_pyr0 + k_pyr_resize x (L-1) read every level l-1 back from HBM to build level l.  Here one
// 1024-thread workgroup per frame walks down the frame once: each round loads the next K0
// level-0 rows into an LDS ring (prefetched into registers during the previous round), and
// every level l >= 1 computes the rows whose two source rows of level l-1 are already in that
// level's ring, writing them to the padded pyramid and (for the next level) to its own ring.
// Level l works on rows its source finished in an earlier round (level 1 on the level-0 rows of
// this round), so all levels run in one task pool per round: two barriers per round, no
// intermediate level ever leaves the CU except as the pyramid itself.  HBM traffic = the input
// read once + every padded level written once.
// The task loop issues no global load: on CDNA the vector-memory counter also counts stores, so
// a table load after a row's stores would wait for them.  The per-column taps live in LDS
// for the whole kernel, and the row entries of round n+1 are staged with the level-0 prefetch.
// The round schedule, ring capacities (the oldest row any round still reads to the newest one
// written by then), ring slots of every row and the per-column resize taps are host-built
// (build_stream_plan); the arithmetic per padded pixel is k_pyr0's / k_pyr_resize's exactly.
// Every ROI row r of a level goes to padded row r + 16 and to its reflect-101 mirrors 16 - r
// (1 <= r <= 16) and 2h + 14 - r (h - 17 <= r <= h - 2); the host requires h, w >= 17.
struct StreamLevel {
    int nq;             // tasks per row: 16-B chunks (level 0) / 4-px quads (l >= 1) of the padded row
    uint32_t nqm;       // ceil(2^32 / nq): row = umulhi(task, nqm) (exact for the task counts used)
    int ringOff;        // LDS byte offset of the level's ring of ROI rows (levels < L-1)
    int ringPitch;      // its row pitch (bytes, multiple of 16)
    int colOff;         // LDS byte offset of the level's column words (l >= 1; 16 B per quad)
    int waveStart, nWaves;  // the workgroup's waves that build this level
    int w, h, pitch;
    long long base, fstride;
};
struct StreamGeom {
    int L, nRounds;
    int u0;             // 16-B units per level-0 ROI row
    uint32_t u0m;       // ceil(2^32 / u0)
    int align;          // input alignment: 16 / 4 / 1 (pointer, stride and frame pitch)
    int colWords;       // u32 column words of all levels (LDS-resident)
    int colOff;         // LDS byte offset of the column words
    int rowOff;         // LDS byte offset of the two row-entry stages (rowStride uint2 each)
    int rowStride;      // row entries per stage (the most any round has)
    int cap0;           // level-0 ring rows (row r in slot r % cap0)
};
#define PS_THREADS 1024
#ifndef PS_LOADERS
#define PS_LOADERS 2  // loader waves per workgroup
#endif
#define PS_NPF 8     // level-0 units (and row entries) per loader lane and round: K0 * u0 <= 1024
#ifndef KR_STREAM_BATCH  // smallest batch that uses k_pyr_stream (one workgroup per frame)
#define KR_STREAM_BATCH 256
#endif
#ifndef PS_LDS_TARGET
#define PS_LDS_TARGET (76 * 1024)  // two workgroups per CU
#endif

// One 16-B unit of a level-0 input row (nvalid >= 1 bytes of it inside the row; bytes past the
// row come back 0).  Aligned input: one 16-B load.  Otherwise (a 1241-px KITTI frame, a pitched
// view, a row's partial last unit): the one or two 16-B-aligned blocks holding the unit's valid
// bytes and a funnel shift — 16 byte loads per unit before, KITTI k_pyr_stream 0.799 -> 0.568 ms
// per 512 frames.  Only blocks holding a valid byte are read (the second is block 0 again when
// not needed, and its bytes are then never used), so no load leaves the pages of the input.
__device__ __forceinline__ uint4 load_unit16(const uint8_t* p, int nvalid, int align) {
    if (nvalid >= 16 && align == 16) return *(const uint4*)p;
    const int sh = (int)((uintptr_t)p & 15u), need = min(nvalid, 16);
    const uint4* blk = (const uint4*)(p - sh);  // pointer arithmetic on p: global, not flat, loads
    const uint4 lo = blk[0];
    const uint4 hi = blk[sh + need > 16 ? 1 : 0];
    // dwords w[d .. d + 4] of the 32-B pair, d = sh >> 2, selected without indexing
    const int d = sh >> 2;
    const uint32_t w0 = lo.x, w1 = lo.y, w2 = lo.z, w3 = lo.w, w4 = hi.x, w5 = hi.y, w6 = hi.z, w7 = hi.w;
    auto pick = [&](int j) {  // w[d + j], 0 <= j <= 4
        const int i = d + j;
        return i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : i == 3 ? w3 : i == 4 ? w4 : i == 5 ? w5 : i == 6 ? w6 : w7;
    };
    const uint32_t s0 = pick(0), s1 = pick(1), s2 = pick(2), s3 = pick(3), s4 = pick(4);
    const uint32_t bs = (uint32_t)(sh & 3);
    uint32_t o[4] = {__builtin_amdgcn_alignbyte(s1, s0, bs), __builtin_amdgcn_alignbyte(s2, s1, bs),
                     __builtin_amdgcn_alignbyte(s3, s2, bs), __builtin_amdgcn_alignbyte(s4, s3, bs)};
    if (need < 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int nb = min(max(need - 4 * q, 0), 4);
            o[q] &= nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        }
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

typedef unsigned short ps_u16x2 __attribute__((ext_vector_type(2)));
// high 32 bits of the 48-bit product of two 24-bit operands (v_mul_hi_u32_u24)
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
}
// LDS-only barrier: the ring and stage hand-offs are LDS; the pyramid stores need not drain
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

#ifndef PS_TIMING  // 1: per-phase s_memtime sums of k_pyr_stream's waves (experiment builds only)
#define PS_TIMING 0
#endif
#if PS_TIMING
__device__ unsigned long long g_pstime[32];
#define PS_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define PS_T(v)
#endif
// rounds[n]: per level lo | cnt << 12 | (first stage entry) << 18 (L words), then the round's
// first row entry in rowEntries and the round's entry count
#ifndef PS_WAVES
#define PS_WAVES 8  // waves per SIMD the register allocation targets (two workgroups per CU)
#endif
#define PS_LB 4  // level-0 units per loader lane in flight at once
#if ORB_ILP_HERE
__global__ void __launch_bounds__(PS_THREADS) __attribute__((amdgpu_waves_per_eu(PS_WAVES)))
k_pyr_stream(const uint8_t* __restrict__ imgs, int stride, long long fpitch, uint8_t* __restrict__ pyr,
             const uint32_t* __restrict__ colWords, const uint4* __restrict__ rowEntries,
             const StreamLevel* __restrict__ slv, const uint32_t* __restrict__ rounds, StreamGeom sg,
             int* __restrict__ cellCount, int nCells) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_ring[];
    const int b = blockIdx.x, tid = threadIdx.x;
    // the frame's per-cell FAST counters for k_fast (when this launch is followed by the rest of
    // the extraction: one memset launch fewer)
    if (cellCount)
        for (int i = tid; i < nCells; i += PS_THREADS) cellCount[(long long)b * nCells + i] = 0;
    const int rw = sg.L + 2;  // words per round record
    for (int i = tid; i < sg.colWords; i += PS_THREADS) ((uint32_t*)(s_ring + sg.colOff))[i] = colWords[i];
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // The first PS_LOADERS waves are loaders: during round n they bring the level-0 rows and
    // the row entries of round n+1 into the ring (whose capacity covers one round ahead) and
    // the other stage, while every other wave builds its level's rows of round n; one barrier
    // per round hands both over.  Builder waves hold no prefetch registers.
    if (wave < PS_LOADERS) {
        const uint8_t* img = imgs + (long long)b * fpitch;
        const int w0 = slv[0].w, r0Off = slv[0].ringOff, r0Pitch = slv[0].ringPitch;
        for (int n = 0; n <= sg.nRounds; ++n) {
            if (n < sg.nRounds) {
                const uint32_t e = rounds[n * rw];
                const int lo = e & 0xFFF, units = (int)((e >> 12) & 0x3F) * sg.u0;
                for (int i0 = tid; i0 < units; i0 += PS_LB * 64 * PS_LOADERS) {
                    uint4 pf[PS_LB];
#pragma unroll
                    for (int k = 0; k < PS_LB; ++k) {
                        const int i = i0 + k * 64 * PS_LOADERS;
                        if (i < units) {
                            const int r = (int)__umulhi((uint32_t)i, sg.u0m), u = i - r * sg.u0;
                            pf[k] = load_unit16(img + (long long)(lo + r) * stride + 16 * u, w0 - 16 * u, sg.align);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < PS_LB; ++k) {
                        const int i = i0 + k * 64 * PS_LOADERS;
                        if (i < units) {
                            const int r = (int)__umulhi((uint32_t)i, sg.u0m), u = i - r * sg.u0;
                            *(uint4*)(s_ring + r0Off + ((lo + r) % sg.cap0) * r0Pitch + 16 * u) = pf[k];
                        }
                    }
                }
            }
            lds_barrier();  // round n's data is in LDS (n = 0: before the first round)
        }
        return;
    }
    // builder waves: this wave's level (host-assigned wave groups) and its column units
    int myL = 0;
    for (int l = 0; l < sg.L; ++l)
        if (wave >= slv[l].waveStart && wave < slv[l].waveStart + slv[l].nWaves) myL = l;
    const int ws = slv[myL].waveStart, nWaves = slv[myL].nWaves;
    const bool idle = wave < ws || wave >= ws + nWaves;  // a wave no level needed
    const int nq = slv[myL].nq, w = slv[myL].w, colOff = slv[myL].colOff;
    uint8_t* D = pyr + slv[myL].base + (long long)b * slv[myL].fstride;
    const int ql = (wave - ws) * 64 + lane, qs = 64 * nWaves;
    // a level >= 1 column quad: its four columns' source offsets, weights and flags
    struct QuadCols {
        int sx[4];
        uint32_t ap[4], live;  // ap = a0 | a1 << 16 (v_dot2 operand)
        uint32_t simd;
        bool allSimd;
        uint32_t hmask;
        uint32_t simdBytes;  // 0xFF in the byte of every SSE2 column (the others: the scalar tail)
    };
    auto decode_quad = [&](const uint4 cw) {
        // column words: sx | a1 << 12 | (a0 - 2047 + a1) << 24 | simd << 26 | live << 27
        QuadCols Q;
        const uint32_t cc[4] = {cw.x, cw.y, cw.z, cw.w};
        Q.live = 0;
        Q.simd = 0;
        Q.simdBytes = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            Q.sx[j] = (int)(cc[j] & 0xFFFu);
            const uint32_t a1 = (cc[j] >> 12) & 0xFFFu;
            Q.ap[j] = (2047u + ((cc[j] >> 24) & 3u) - a1) | (a1 << 16);
            if (cc[j] & (1u << 26)) Q.simd |= 1u << j, Q.simdBytes |= 0xFFu << (8 * j);
            if (cc[j] & (1u << 27)) Q.live |= 0xFFu << (8 * j);
        }
        Q.allSimd = Q.simd == 0xFu;
        Q.hmask = Q.allSimd ? 0xFFFFFFF0u : 0xFFFFFFFFu;  // (H >> 4) << 4 on all-SSE2 quads
        return Q;
    };
    auto build_quad = [&](const int q, const QuadCols& Q, const uint4* E, const int cnt) {
        const int* sx = Q.sx;
        const uint32_t* ap = Q.ap;
        const uint32_t live = Q.live, hmask = Q.hmask;
        const bool allSimd = Q.allSimd;
        // the level's scalar-tail columns (VResizeLinear's columns past the SSE2 body: one or two
        // quads per level) make their wave take the mixed path below for every row; the other
        // waves run the all-SSE2 formula alone (wave-uniform: no divergent path per row)
        const bool waveTail = __ballot(!allSimd) != 0ull;
        const uint32_t simdBytes = Q.simdBytes;
        // HResizeLinear of the source row at LDS address `ra`: H = S[sx] a0 + S[sx+1] a1
        // (a1 == 0 where OpenCV reads S[sx] only: the byte after it is multiplied by 0; it
        // lies in the ring row's slack or the next LDS row, never outside the allocation).
        // On all-SSE2 quads h keeps (H >> 4) << 4 = H & ~15 for the v_mul_hi_u32_u24 below.
        auto hrow = [&](uint32_t ra, uint32_t* hh) {
            const uint8_t* R = s_ring + ra;
            uint32_t lo8[4], hi8[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lo8[j] = R[sx[j]];
                hi8[j] = R[sx[j] + 1];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t H = __builtin_amdgcn_udot2(__builtin_bit_cast(ps_u16x2, lo8[j] | (hi8[j] << 16)),
                                                          __builtin_bit_cast(ps_u16x2, ap[j]), 0u, false);
                hh[j] = H & hmask;
            }
        };
        const int cx = 4 * q - EDGE;
        const bool roi = cx >= 0 && cx < w;
        // one output row from its two source rows' horizontal sums hA (row s0) and hB (row s1)
        auto vrow = [&](const uint4 e0, const uint4 e1, const uint32_t* hA, const uint32_t* hB) {
            uint32_t word = 0;
            if (!waveTail) {
                // VResizeLinearVec_32s8u: ((H >> 4) * b) >> 16 per term = the high 32 bits of
                // (H & ~15) * (b << 12) (both < 2^24), + 2 >> 2
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    word |= ((mulhi24(hA[j], e0.z) + mulhi24(hB[j], e0.w) + 2u) >> 2) << (8 * j);
            } else {
                // both formulas for every column, the byte per column by one v_bfi (the branchy
                // per-column select cost the tail's wave both paths every row: k_pyr_stream 316 ->
                // 284 us c3 without it, timing-only ablation): SSE2 on H & ~15 (a tail quad's sums
                // are unmasked), the scalar VResizeLinear (H0 b0 + H1 b1 + 2^21) >> 22 on H
                const uint32_t b0 = e0.z >> 12, b1 = e0.w >> 12;
                uint32_t ws = 0, wc = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    ws |= ((mulhi24(hA[j] & ~15u, e0.z) + mulhi24(hB[j] & ~15u, e0.w) + 2u) >> 2) << (8 * j);
                    wc |= ((__umul24(hA[j], b0) + __umul24(hB[j], b1) + (1u << 21)) >> 22) << (8 * j);
                }
                word = bfi(simdBytes, ws, wc);
            }
            word &= live;
            // wave-uniform row base (SGPRs) + the lane's 32-bit offset: no 64-bit VALU address
            // add per store and row (nothing in this kernel reads the pyramid back)
            const uint32_t qo = 4u * (uint32_t)q;
            auto store_row = [&](uint32_t off) {
                asm volatile("global_store_dword %0, %1, %2" ::"v"(qo), "v"(word), "s"(D + off) : "memory");
            };
            store_row(e1.y);
            if (e1.z != 0xFFFFFFFFu) store_row(e1.z);
            if (e1.w != 0xFFFFFFFFu) store_row(e1.w);
            if (e1.x != 0xFFFFFFFFu && roi) *(uint32_t*)(s_ring + e1.x + cx) = word;
        };
        // Rows in pairs with the source roles alternating: even rows read (hP, hQ), odd rows
        // (hQ, hP).  A downscale step's next row starts at this row's second source row (held
        // in the set the next row reads first), so only the other set is recomputed, and no
        // row ever copies sums between register sets.  (tP / tQ: the rows they hold.)
        uint32_t tP = 0xFFFFFFFFu, tQ = 0xFFFFFFFFu;
        uint32_t hP[4] = {0u, 0u, 0u, 0u}, hQ[4] = {0u, 0u, 0u, 0u};
        for (int k = 0; k < cnt; k += 2) {
            {
                const uint4 e0 = E[2 * k], e1 = E[2 * k + 1];
                if (tP != e0.x) hrow(e0.x, hP), tP = e0.x;
                if (tQ != e0.y) hrow(e0.y, hQ), tQ = e0.y;
                vrow(e0, e1, hP, hQ);
            }
            if (k + 1 < cnt) {
                const uint4 e0 = E[2 * k + 2], e1 = E[2 * k + 3];
                if (tQ != e0.x) hrow(e0.x, hQ), tQ = e0.x;
                if (tP != e0.y) hrow(e0.y, hP), tP = e0.y;
                vrow(e0, e1, hQ, hP);
            }
        }
    };
    // a level whose quads fit one pass of its waves (every level of 640-px frames): each lane's
    // quad decoded once for the whole kernel instead of once per round
    const bool hoisted = myL > 0 && !idle && nq <= qs;
    lds_barrier();  // the column words are in LDS
    QuadCols col0{};
    if (hoisted) col0 = decode_quad(((const uint4*)(s_ring + colOff))[min(ql, nq - 1)]);
#if PS_TIMING
    unsigned long long acc[5] = {0, 0, 0, 0, 0};
#endif
    for (int n = 0; n < sg.nRounds; ++n) {
        PS_T(t1);
        const uint32_t e = idle ? 0u : rounds[n * rw + myL];
        const int cnt = (e >> 12) & 0x3F;
        // the level's row entries of this round (scalar loads: lgkmcnt, never behind stores):
        // {source row 0, source row 1 (LDS addresses), b0 << 12, b1 << 12, own ring row (LDS
        //  address, ~0u: none), padded-row offset, top mirror offset, bottom mirror offset (~0u: none)}
        const uint4* E = rowEntries + 2 * ((int)rounds[n * rw + sg.L] + (int)(e >> 18));
        if (cnt > 0 && myL == 0) {
            // padded level-0 rows from the ring (k_pyr0's copyMakeBorder), 16 B per unit
            for (int c = ql; c < nq; c += qs) {
                const int px = 16 * c;
                const bool inner = px >= EDGE && px <= w;
                for (int k = 0; k < cnt; ++k) {
                    const uint4 e0 = E[2 * k], e1 = E[2 * k + 1];
                    const uint8_t* R = s_ring + e0.x;
                    uint4 v;
                    if (inner) {
                        v = *(const uint4*)(R + px - EDGE);
                    } else if (px == 0) {
                        // left border: bytes R[16], R[15], .. R[1] (reflect-101 of -16 .. -1),
                        // the aligned dwords R[0..19] reversed by v_perm
                        const uint4 a = *(const uint4*)R;
                        const uint32_t a4 = *(const uint32_t*)(R + 16);
                        v = make_uint4(__builtin_amdgcn_perm(a4, a.w, 0x01020304u), __builtin_amdgcn_perm(a.w, a.z, 0x01020304u),
                                       __builtin_amdgcn_perm(a.z, a.y, 0x01020304u), __builtin_amdgcn_perm(a.y, a.x, 0x01020304u));
                    } else if ((w & 15) == 0 && px == w + EDGE) {
                        // right border of a 16-aligned row: R[w-2], R[w-3], .. R[w-17], from the
                        // aligned dwords R[w-32 .. w-1] (E0 .. E7) reversed by v_perm
                        const uint4 lo = *(const uint4*)(R + w - 32), hi = *(const uint4*)(R + w - 16);
                        v = make_uint4(__builtin_amdgcn_perm(hi.w, hi.z, 0x03040506u), __builtin_amdgcn_perm(hi.z, hi.y, 0x03040506u),
                                       __builtin_amdgcn_perm(hi.y, hi.x, 0x03040506u), __builtin_amdgcn_perm(hi.x, lo.w, 0x03040506u));
                    } else {  // a border unit: single-bounce reflect-101 (w >= 17); all 16
                              // reads unconditional (clamped), so they issue back to back.  (The
                              // compiler hoists the 16 indices out of the row loop for every unit;
                              // keeping them in this branch measured slower: the border lanes share
                              // the level-0 wave, which then ran them for every row, 0.394 vs
                              // 0.380 ms c3)
                        const int pxo = px;
                        uint32_t by[16];
#pragma unroll
                        for (int j = 0; j < 16; ++j) {
                            const int X = min(pxo + j - EDGE, w + EDGE - 1);
                            by[j] = R[X < 0 ? -X : (X >= w ? 2 * w - 2 - X : X)];
                        }
                        uint32_t w4[4];
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4) {
                            uint32_t word = 0;
#pragma unroll
                            for (int j = 0; j < 4; ++j) word |= (pxo + 4 * q4 + j < w + 2 * EDGE ? by[4 * q4 + j] : 0u) << (8 * j);
                            w4[q4] = word;
                        }
                        v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                    }
                    *(uint4*)(D + e1.y + px) = v;
                    if (e1.z != 0xFFFFFFFFu) *(uint4*)(D + e1.z + px) = v;
                    if (e1.w != 0xFFFFFFFFu) *(uint4*)(D + e1.w + px) = v;
                }
            }
        } else if (cnt > 0) {
            // level myL from the ring of level myL-1: per column unit, the round's rows in order
            if (hoisted) {
                if (ql < nq) build_quad(ql, col0, E, cnt);
            } else {
                const uint4* C = (const uint4*)(s_ring + colOff);
                for (int q = ql; q < nq; q += qs) build_quad(q, decode_quad(C[q]), E, cnt);
            }
        }
        PS_T(t2);
        lds_barrier();
#if PS_TIMING
        PS_T(t3);
        acc[1] += t2 - t1;
        acc[2] += t3 - t2;
#endif
    }
#if PS_TIMING
    if (lane == 0) {
        for (int k = 0; k < 5; ++k) atomicAdd(&g_pstime[k], acc[k]);
        atomicAdd(&g_pstime[5], 1ull);
        if (!idle) {
            atomicAdd(&g_pstime[8 + myL], acc[1]);
            atomicAdd(&g_pstime[24 + myL], 1ull);
        }
    }
#endif
}
#endif  // ORB_ILP_HERE

typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Compass pre-filter of cv::FAST for the 4 pixels of a dword, in packed 16-bit arithmetic on
// the dword's even and odd bytes (pixels x, x+2 / x+1, x+3) split into u16 lanes by the caller.
// Bright: (q0 > v+t or q8 > v+t) and (q4 or q12 likewise) <=> M = min(max(q0, q8), max(q4, q12))
// > v + t; dark: m = max(min(q0, q8), min(q4, q12)) < v - t; so the pixel passes <=>
// max(M - v, v - m) > t, the sign of t - max(M - v, v - m) (all values within i16).
// Returns a 4-bit mask (bit j = pixel j passes).
__device__ __forceinline__ uint32_t compass_half(uint32_t v, uint32_t q0, uint32_t q4, uint32_t q8, uint32_t q12,
                                                 uint32_t tt) {
    const u16x2 a = __builtin_bit_cast(u16x2, q0), b = __builtin_bit_cast(u16x2, q4);
    const u16x2 d = __builtin_bit_cast(u16x2, q8), e = __builtin_bit_cast(u16x2, q12);
    const i16x2 M = __builtin_bit_cast(
        i16x2, __builtin_elementwise_min(__builtin_elementwise_max(a, d), __builtin_elementwise_max(b, e)));
    const i16x2 m = __builtin_bit_cast(
        i16x2, __builtin_elementwise_max(__builtin_elementwise_min(a, d), __builtin_elementwise_min(b, e)));
    const i16x2 vv = __builtin_bit_cast(i16x2, v);
    const i16x2 X = __builtin_elementwise_max((i16x2)(M - vv), (i16x2)(vv - m));
    return __builtin_bit_cast(uint32_t, (i16x2)(__builtin_bit_cast(i16x2, tt) - X));  // bit 15 / 31: passes
}
__device__ __forceinline__ uint32_t compass_mask(uint32_t pe, uint32_t po) {
    // bit 15 / 31 of even -> pixels 0 / 2, of odd -> pixels 1 / 3: bytes (even 1, odd 1, even 3,
    // odd 3) gathered by one v_perm, their sign bits to bit 0 of each byte, packed by one v_dot4
    const uint32_t g4 = (__builtin_amdgcn_perm(po, pe, 0x07030501u) >> 7) & 0x01010101u;
    return __builtin_amdgcn_udot4(g4, 0x08040201u, 0u, false);
}
__device__ __forceinline__ uint32_t even_bytes(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c020c00u); }
__device__ __forceinline__ uint32_t odd_bytes(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c030c01u); }
// the pre-filter of one dword from its five words (centre, q0 = 3 rows below, q4 = 3 px right,
// q8 = 3 rows above, q12 = 3 px left)
__device__ __forceinline__ uint32_t compass4(uint32_t c, uint32_t q0, uint32_t q4, uint32_t q8, uint32_t q12,
                                             uint32_t tt) {
    return compass_mask(compass_half(even_bytes(c), even_bytes(q0), even_bytes(q4), even_bytes(q8), even_bytes(q12), tt),
                        compass_half(odd_bytes(c), odd_bytes(q0), odd_bytes(q4), odd_bytes(q8), odd_bytes(q12), tt));
}
#ifndef KR_COMPASS8
#define KR_COMPASS8 1
#endif
// cv::FAST's full pre-test (all eight even circle points): a 9-arc holds a point of every
// antipodal pair {k, k+8}, so bright <=> min over the four pairs of their max > v + t and dark
// <=> max over the pairs of their min < v - t are necessary.  Stronger than compass_half (two
// pairs), for the FAST(7) re-runs whose low threshold lets most noisy pixels through the compass.
__device__ __forceinline__ uint32_t compass8_half(uint32_t v, uint32_t q0, uint32_t q8, uint32_t q4, uint32_t q12,
                                                  uint32_t q2, uint32_t q10, uint32_t q6, uint32_t q14, uint32_t tt) {
    const u16x2 a0 = __builtin_bit_cast(u16x2, q0), a8 = __builtin_bit_cast(u16x2, q8);
    const u16x2 a4 = __builtin_bit_cast(u16x2, q4), a12 = __builtin_bit_cast(u16x2, q12);
    const u16x2 a2 = __builtin_bit_cast(u16x2, q2), a10 = __builtin_bit_cast(u16x2, q10);
    const u16x2 a6 = __builtin_bit_cast(u16x2, q6), a14 = __builtin_bit_cast(u16x2, q14);
    const i16x2 M = __builtin_bit_cast(
        i16x2, __builtin_elementwise_min(
                   __builtin_elementwise_min(__builtin_elementwise_max(a0, a8), __builtin_elementwise_max(a4, a12)),
                   __builtin_elementwise_min(__builtin_elementwise_max(a2, a10), __builtin_elementwise_max(a6, a14))));
    const i16x2 m = __builtin_bit_cast(
        i16x2, __builtin_elementwise_max(
                   __builtin_elementwise_max(__builtin_elementwise_min(a0, a8), __builtin_elementwise_min(a4, a12)),
                   __builtin_elementwise_max(__builtin_elementwise_min(a2, a10), __builtin_elementwise_min(a6, a14))));
    const i16x2 vv = __builtin_bit_cast(i16x2, v);
    const i16x2 X = __builtin_elementwise_max((i16x2)(M - vv), (i16x2)(vv - m));
    return __builtin_bit_cast(uint32_t, (i16x2)(__builtin_bit_cast(i16x2, tt) - X));
}
// the eight-point pre-test of one dword from its centre row (dwords -1, 0, +1: lf, cc, rg), the rows
// 3 below / above (dn, up) and the rows 2 below / above (dwords -1, 0, +1: d2*, u2*)
__device__ __forceinline__ uint32_t compass8(uint32_t lf, uint32_t cc, uint32_t rg, uint32_t dn, uint32_t up,
                                             uint32_t d2l, uint32_t d2c, uint32_t d2r, uint32_t u2l, uint32_t u2c,
                                             uint32_t u2r, uint32_t tt) {
    const uint32_t q4 = __builtin_amdgcn_alignbyte(rg, cc, 3), q12 = __builtin_amdgcn_alignbyte(cc, lf, 1);
    // circle points 2 = (+2, +2), 14 = (+2, -2) on the row 2 below; 6 = (-2, +2), 10 = (-2, -2) 2 above
    const uint32_t q2 = __builtin_amdgcn_alignbyte(d2r, d2c, 2), q14 = __builtin_amdgcn_alignbyte(d2c, d2l, 2);
    const uint32_t q6 = __builtin_amdgcn_alignbyte(u2r, u2c, 2), q10 = __builtin_amdgcn_alignbyte(u2c, u2l, 2);
    return compass_mask(compass8_half(even_bytes(cc), even_bytes(dn), even_bytes(up), even_bytes(q4), even_bytes(q12),
                                      even_bytes(q2), even_bytes(q10), even_bytes(q6), even_bytes(q14), tt),
                        compass8_half(odd_bytes(cc), odd_bytes(dn), odd_bytes(up), odd_bytes(q4), odd_bytes(q12),
                                      odd_bytes(q2), odd_bytes(q10), odd_bytes(q6), odd_bytes(q14), tt));
}

// ---- FAST strength --------------------------------------------------------------------------
// S(p) = 1 + cornerScore<16>(p) of cv::FAST: the largest t for which p is a corner is S - 1,
// so p is a corner at threshold t <=> S > t; records carry S - 1 as the score.
// Both sides in one packed register of two exact f16 values: lane 0 carries the dark
// contrast v - c, lane 1 the bright contrast c - v, as multiples of 2^-24 (a byte b loaded
// into a VGPR is the f16 denormal b * 2^-24, so the pair is one v_pk_add_f16 of the two
// loaded bytes, no packing; all values are integers in [-255, 255] times 2^-24, exact).  Arcs
// of 9 as windows of 3 (two v_pk_minimum3_f16 per arc, gfx950), the best arc by
// v_pk_maximum3_f16: ~45 VALU per pixel (round 2's 1024 + b normal encoding needed a shift and
// an or per circle pixel before the add: ~75; the i16 version ~150).  Cheap enough to
// run on every pre-filter survivor instead of a 9-arc test followed by a second gather for the
// corners (k_fast's queue is LDS-latency bound).
#ifndef FS_I16  // 1: the previous i16 arithmetic (experiments)
#define FS_I16 0
#endif
typedef short s16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int fast_strength_packed(const uint8_t* p, int TP) {
    const uint32_t v = p[0];
#if FS_I16
    const int off[16] = {3 * TP, 3 * TP + 1, 2 * TP + 2, TP + 3, 3, -TP + 3, -2 * TP + 2, -3 * TP + 1,
                         -3 * TP, -3 * TP - 1, -2 * TP - 2, -TP - 3, -3, TP - 3, 2 * TP - 2, 3 * TP - 1};
    s16x2_t d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t c = p[off[k]];
        // (v, c) - (c, v) = (v - c, c - v)
        d[k] = __builtin_bit_cast(s16x2_t, v | (c << 16)) - __builtin_bit_cast(s16x2_t, c | (v << 16));
    }
    s16x2_t m2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m2[k] = __builtin_elementwise_min(d[k], d[(k + 1) & 15]);
    s16x2_t best;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const s16x2_t w9 = __builtin_elementwise_min(
            __builtin_elementwise_min(__builtin_elementwise_min(m2[k], m2[(k + 2) & 15]),
                                      __builtin_elementwise_min(m2[(k + 4) & 15], m2[(k + 6) & 15])),
            d[(k + 8) & 15]);
        best = k ? __builtin_elementwise_max(best, w9) : w9;
    }
    return max((int)best.x, (int)best.y);
#else
    // a byte b read into a VGPR is the f16 denormal b * 2^-24: (v - c, c - v) is one v_pk_add_f16
    // of the two loaded bytes with both lanes on the low halves and one side negated per lane
    // (exact: differences of denormals are exact; f16 denormals are not flushed).  The circle's
    // bytes are read from one base per row (rows y-3 .. y+3, from column x-3) with the column as
    // the ds_read immediate: seven address adds instead of one per circle point
    constexpr int kDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    constexpr int kDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    // (the base column x-3 made opaque: the compiler otherwise re-derives the bases from p and
    // adds the negative column offsets separately, DS offsets being unsigned)
    typedef const __attribute__((address_space(3))) uint8_t* lds_u8p;
    uint32_t a0 = (uint32_t)(uintptr_t)(lds_u8p)p - 3u;
    asm volatile("" : "+v"(a0));
    lds_u8p rowp[7];
#pragma unroll
    for (int r = 0; r < 7; ++r) rowp[r] = (lds_u8p)(uintptr_t)(a0 + (uint32_t)((r - 3) * TP));
    f16x2_t d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t c = rowp[kDy[k] + 3][kDx[k] + 3];
        uint32_t r;
        asm("v_pk_add_f16 %0, %1, %2 op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(r) : "v"(v), "v"(c));
        d[k] = __builtin_bit_cast(f16x2_t, r);
    }
    f16x2_t m3[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    f16x2_t best = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[0], m3[3]), m3[6]);
#pragma unroll
    for (int k = 1; k < 16; k += 2) {
        const f16x2_t a = __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
        const f16x2_t c = k + 1 < 16 ? __builtin_elementwise_minimum(__builtin_elementwise_minimum(m3[k + 1], m3[(k + 4) & 15]), m3[(k + 7) & 15]) : a;
        best = __builtin_elementwise_maximum(__builtin_elementwise_maximum(best, a), c);
    }
    // back to integers: a positive denormal's bits are its value; a negative one (or -0) is a
    // negative i16 (sign bit set), and S <= 0 is no corner at any threshold >= 0
    const uint32_t bb = __builtin_bit_cast(uint32_t, best);
    return max((int)(short)(bb & 0xFFFFu), (int)(short)(bb >> 16));
#endif
}

// The reference's `FAST(cellImage, keys, 7, true)` re-run of a cell that kept <= 3 corners at
// fastTh (ORBextractor.cc:609-614), by a whole 256-thread workgroup: the cell ROI with its
// 3 px ring is staged into LDS with 16-byte loads, the strength plane at t = 7 computed, 3x3
// strict NMS inside the detection region (out-of-region neighbours 0, as cv::FAST on the cell
// Mat), survivors written in raster order as ((S - 1) << 24) | (y << 12) | x.  Returns the
// survivor count (all threads).  smem: Sp (dwp x dh, 16-B padded) | Bm (dh x bw survivor mask
// words) | rowc | In (the ROI staged from its 16-B aligned start with 16-B loads: the dword
// staging before needed 128 VGPRs for its 20 loads in flight per thread, 4 waves per SIMD; 16-B
// units need 50: re-runs 0.174 -> 0.123 ms per 512 KITTI frames, 2.61 -> 2.02 per 4096 720p),
// rerun_lds() bytes.  Output: each survivor sets its bit in its row's mask
// and counts into its row; after the row prefix one thread per mask word writes that word's
// survivors at the row's offset + the set bits of the row's earlier words (no per-row scan of
// the cell, no list, no returning atomics in the NMS).
#define RR_Q 320  // per-wave queue of compass survivors (< 64 carried + 4 x 64 new), + a trash slot
inline size_t rerun_lds(int dw, int dh) {
    const size_t dwp = (size_t)((dw + 3) & ~3);
    const size_t inW = (size_t)((15 + dw + 6 + 15) & ~15), spBytes = (dwp * dh + 15) & ~(size_t)15;
    const size_t bmBytes = 4 * (size_t)((dh * ((dw + 31) >> 5) + 3) & ~3);
    return spBytes + bmBytes + 4 * (size_t)((dh + 3) & ~3) + inW * (dh + 6) + 16 + 4 * (4 + 4 * (RR_Q + 8));
}
// Stage `rows` x `units` 16-B units (global row pitch gsu units) into LDS (row pitch = units):
// SB4 units per thread per batch, all loads of a batch in flight before any LDS write
template <int NT, int SB4>
__device__ __forceinline__ void stage_units_to_lds(uint4* __restrict__ dst, const uint4* __restrict__ src, long long gsu,
                                                   int rows, int units, int tid) {
    const int total = rows * units;
    const int dr = NT / units, dc = NT - dr * units;
    for (int base = 0; base < total; base += SB4 * NT) {
        const int i0 = base + tid;
        const int r0 = i0 / units, c0 = i0 - r0 * units;
        uint4 v[SB4];
        int r = r0, c = c0;
#pragma unroll
        for (int k = 0; k < SB4; ++k) {
            const bool ok = base + k * NT + tid < total;
            v[k] = src[ok ? (long long)r * gsu + c : 0ll];
            r += dr;
            c += dc;
            if (c >= units) {
                c -= units;
                ++r;
            }
        }
#pragma unroll
        for (int k = 0; k < SB4; ++k)
            if (base + k * NT + tid < total) dst[base + k * NT + tid] = v[k];
    }
}
__device__ int cell_fast_rerun(const uint8_t* __restrict__ det, int pitch, int dw, int dh, int rx0, int ry0, int t,
                               uint8_t* smem, uint32_t* __restrict__ out, int tid, int level) {
    const int wave = tid >> 6, lane = tid & 63;
    KR_T(0);
    const int dwp = (dw + 3) & ~3, rw = dwp >> 2, nw = (dh * dwp) >> 2;
    uint8_t* Sp = smem;
    const int spWords = ((dh * dwp + 15) & ~15) >> 2;  // In stays 16-B aligned
    uint32_t* Bm = (uint32_t*)Sp + spWords;  // survivor bits, bw words per row
    const int bw = (dw + 31) >> 5;
    const int bmWords = (dh * bw + 3) & ~3;
    int* rowc = (int*)(Bm + bmWords);
    uint8_t* In = (uint8_t*)(rowc + ((dh + 3) & ~3));
    const int o = (int)((uintptr_t)(det - 3) & 15);  // 16-B alignment of the staged ROI
    const int inW = (o + dw + 6 + 15) & ~15;
    {
        // 16-B units from the aligned start (the pitch is a multiple of 16; the over-read stays
        // in the row's padding or the next row, and its bytes are never used)
        const uint4* src = (const uint4*)(det - 3 * (long long)pitch - 3 - o);
        stage_units_to_lds<256, 4>((uint4*)In, src, pitch >> 4, dh + 6, inW >> 4, tid);
        // Sp and Bm's area (contiguous from the 16-B aligned smem) zeroed with 16-B stores: a
        // pixel the compass rejects keeps strength 0
        const int nz = spWords + bmWords;
        const int z16 = nz >> 2;
        for (int i = tid; i < z16; i += 256) ((uint4*)Sp)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = 4 * z16 + tid; i < nz; i += 256) ((uint32_t*)Sp)[i] = 0u;
        for (int i = tid; i < dh; i += 256) rowc[i] = 0;
    }
    __syncthreads();
    KR_T(1);
    // the strength plane (corner at t <=> S > t; the NMS below reads only S > t, so a pixel
    // known not to be a corner may hold 0): per wave, 64 staged dwords (4 pixels each) at a
    // time through the compass test of cv::FAST at t in packed 16-bit arithmetic (compass4, as
    // k_fast: a 9-arc always covers two cyclically adjacent points of {0, 4, 8, 12}, a
    // necessary condition), survivors queued as pixel indices, the exact strength computed in
    // full 64-lane passes from the top of the queue (LDS accesses of one wave complete in order)
    {
        uint32_t* q = (uint32_t*)(In + inW * (dh + 6)) + 4 + wave * (RR_Q + 8);  // after the staged ROI
        // i / d = umulhi(i, ceil(2^32 / d)) for d >= 2 (the reciprocal of 1 does not fit 32 bits)
        const uint32_t m = (uint32_t)((0x100000000ull + dw - 1) / (uint64_t)dw);
        // staged dword columns holding detection pixels: In byte c = xx + 3 + o, xx in [0, dw)
        const int wd0 = (3 + o) >> 2, nd = ((dw + 2 + o) >> 2) - wd0 + 1;
        const uint32_t md = (uint32_t)((0x100000000ull + nd - 1) / (uint64_t)nd);
        const int total = dh * nd, iw = inW >> 2;
        const uint32_t tt = (uint32_t)t | ((uint32_t)t << 16);
        const uint32_t* In32 = (const uint32_t*)In;
        int np = 0;
        auto pass = [&](int base, int n) {  // q[base .. base + n), n <= 64
            if (lane < n) {
                const int i = q[base + lane];
                const int yy = dw > 1 ? (int)__umulhi((uint32_t)i, m) : i, xx = i - yy * dw;
                const int S = fast_strength_packed(In + (yy + 3) * inW + xx + 3 + o, inW);
                Sp[yy * dwp + xx] = (uint8_t)(S > t ? S : 0);  // only corners at t carry a strength
            }
        };
        // one strength call site (the last round flushes the queue's remainder)
        for (int i0 = wave * 64;; i0 += 256) {
            const bool last = i0 >= total;  // wave-uniform
            if (!last) {
                const int i = i0 + lane;
                uint32_t mask = 0u;
                int px0 = 0;
                if (i < total) {
                    const int yy = nd > 1 ? (int)__umulhi((uint32_t)i, md) : i, wd = wd0 + i - yy * nd;
                    const uint32_t* row = In32 + (yy + 3) * iw + wd;
                    const uint32_t cc = row[0], lf = row[-1], rg = row[1], up = row[-3 * iw], dn = row[3 * iw];
                    const int xx0 = 4 * wd - 3 - o;  // detection column of byte 0
                    const int lo = max(0, -xx0), hi = min(4, dw - xx0);
                    const uint32_t cols = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
#if KR_COMPASS8
                    const uint32_t* d2 = row + 2 * iw;
                    const uint32_t* u2 = row - 2 * iw;
                    mask = compass8(lf, cc, rg, dn, up, d2[-1], d2[0], d2[1], u2[-1], u2[0], u2[1], tt) & cols;
#else
                    mask = compass4(cc, dn, __builtin_amdgcn_alignbyte(rg, cc, 3), up,
                                    __builtin_amdgcn_alignbyte(cc, lf, 1), tt) & cols;
#endif
                    px0 = yy * dw + xx0;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool c = (mask >> j) & 1u;
                    const uint64_t bm = __ballot(c);
                    q[select_by_mask(bm, RR_Q, np + lanes_below(bm))] = (uint32_t)(px0 + j);  // RR_Q: trash slot
                    np += __popcll(bm);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            while (np >= 64 || (last && np > 0)) {
                const int n = min(np, 64);
                np -= n;
                pass(np, n);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (last) break;
        }
    }
    __syncthreads();
    KR_T(2);
    // 3x3 NMS on the corners only: Sp holds S where S > t and 0 elsewhere, so cv::FAST's strict
    // test s0 - 1 > (n > t ? n - 1 : 0) reads the plane as is (out-of-cell neighbours 0).  Each
    // wave scans its share of the plane's dwords, ballot-compacts the nonzero pixels into its
    // queue (the strength pass is done with it) and runs the NMS one corner per lane, all nine
    // reads issued together; a survivor sets its bit in its row's mask and counts into its row
    // (LDS atomics); the per-word pass below turns the masks into raster-order records
    {
        uint32_t* q = (uint32_t*)(In + inW * (dh + 6)) + 4 + wave * (RR_Q + 8);
        const uint32_t* Sp32 = (const uint32_t*)Sp;
        const uint32_t mr = rw > 1 ? (uint32_t)((0x100000000ull + rw - 1) / (uint64_t)rw) : 0u;
        auto nms = [&](int n) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int k0 = 0; k0 < n; k0 += 64) {
                if (k0 + lane < n) {
                    const uint32_t code = q[k0 + lane];
                    const int yy = (int)(code >> 16), xx = (int)(code & 0xFFFFu);
                    const uint8_t* sp = Sp + yy * dwp + xx;
                    const int s0 = sp[0];
                    const bool xl = xx > 0, xr = xx + 1 < dw, yu = yy > 0, yd = yy + 1 < dh;
                    const int n0 = (yu && xl) ? sp[-dwp - 1] : 0, n1 = yu ? sp[-dwp] : 0, n2 = (yu && xr) ? sp[-dwp + 1] : 0;
                    const int n3 = xl ? sp[-1] : 0, n4 = xr ? sp[1] : 0;
                    const int n5 = (yd && xl) ? sp[dwp - 1] : 0, n6 = yd ? sp[dwp] : 0, n7 = (yd && xr) ? sp[dwp + 1] : 0;
                    const int m = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
                    if (s0 > m) {  // s0 > t: a stored strength
                        atomicOr(&Bm[yy * bw + (xx >> 5)], 1u << (xx & 31));
                        atomicAdd(&rowc[yy], 1);
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        };
        int cn = 0;
        for (int i0 = wave * 64; i0 < nw; i0 += 256) {  // wave-uniform
            const int i = i0 + lane;
            uint32_t w4 = 0u;
            int yy = 0, wd = 0;
            if (i < nw) {
                yy = rw > 1 ? (int)__umulhi((uint32_t)i, mr) : i;
                wd = i - yy * rw;
                w4 = Sp32[i];
            }
            if (__ballot(w4 != 0u) == 0ull) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool v = ((w4 >> (8 * j)) & 0xFFu) != 0u;
                const uint64_t m = __ballot(v);
                q[select_by_mask(m, RR_Q, cn + lanes_below(m))] = ((uint32_t)yy << 16) | (uint32_t)(4 * wd + j);
                cn += __popcll(m);
            }
            if (cn > RR_Q - 256) {
                nms(cn);
                cn = 0;
            }
        }
        if (cn) nms(cn);
    }
    __syncthreads();
    KR_T(3);
    __shared__ int s_total;
    if (wave == 0) {
        int carry = 0;
        for (int r0 = 0; r0 < dh; r0 += 64) {
            const int r = r0 + lane;
            const int v = r < dh ? rowc[r] : 0;
            const int incl = wave_incl_scan(v);
            if (r < dh) rowc[r] = carry + incl - v;
            carry += __builtin_amdgcn_readlane(incl, 63);
        }
        if (lane == 0) s_total = carry;
    }
    __syncthreads();
    const int totalK = s_total;
    // one thread per mask word: its survivors' raster positions start at the row's offset + the
    // set bits of the row's earlier words (each record: the stored strength and the position)
    for (int i = tid; i < dh * bw; i += 256) {
        uint32_t m = Bm[i];
        if (!m) continue;
        const int yy = i / bw, w = i - yy * bw;
        const uint32_t* br = Bm + yy * bw;
        int pos = rowc[yy];
        for (int w2 = 0; w2 < w; ++w2) pos += __popc(br[w2]);
        const uint32_t ly = (uint32_t)(ry0 + yy) << 12;
        while (m) {
            const int xx = 32 * w + __builtin_ctz(m);
            m &= m - 1;
            const uint32_t sc = (uint32_t)(Sp[yy * dwp + xx] - 1);
            out[pos++] = (sc << 24) | ly | (uint32_t)(rx0 + xx);
        }
    }
    __syncthreads();  // smem is reused by the caller
#if KR_TIMING
    // phases: 0 stage + zero, 1 compass + strength, 2 NMS, 3 row scan + output; [4] = cells,
    // [5] = detection pixels, [6] = corners kept
    if (tid == 0) {
        atomicAdd(&g_krtime[level][0], krt1 - krt0);
        atomicAdd(&g_krtime[level][1], krt2 - krt1);
        atomicAdd(&g_krtime[level][2], krt3 - krt2);
        atomicAdd(&g_krtime[level][3], __builtin_amdgcn_s_memrealtime() - krt3);
        atomicAdd(&g_krtime[level][4], 1ull);
        atomicAdd(&g_krtime[level][5], (unsigned long long)(dw * dh));
        atomicAdd(&g_krtime[level][6], (unsigned long long)totalK);
    }
#endif
    return totalK;
}

// The FAST(7) re-runs of every (frame, level), at every batch size, before k_select<.., false>
// (the in-k_select re-run path, k_select<.., true>, is kept only for -DKS_SEP_PIXELS
// experiments): NWG workgroups per (frame, level), workgroup (b * NWG + gw, l)
// re-running the level's fallback cells gw, gw + NWG, ... (in cell order), so one frame's
// re-runs — serial inside k_select's single workgroup per level — spread over many CUs.  A
// cell re-runs where the reference's does: not skipped, and min(count, cap) <= 3 with 0 for a
// cell with no detection area.  The new count is stored with RERUN_FLAG set, so a workgroup
// deciding later still counts the cell among the fallback cells (the ordinal -> workgroup
// assignment is the same everywhere, and so is the decision of every wave of a workgroup).
#ifndef KR_NWG_MIN  // least k_rerun workgroups per (frame, level): at B = 512, 1 / 2 / 3 / 4 measured
#define KR_NWG_MIN 3  // re-runs + selection 640x480 0.146 / 0.117 / 0.116 / 0.132 ms, 1241x376
#endif                // 0.463 / 0.380 / 0.357 / 0.406, 1280x720 0.814 / 0.809 / 0.765 / 0.910
#define RERUN_FLAG 0x40000000
#define COUNT_MASK 0x3FFFFFFF
#ifndef KR_WAVES
#define KR_WAVES 4  // waves per SIMD k_rerun's register allocation targets; re-runs + selection at
                    // B = 512 with 2 / 3 / 5 / 6 / 8: 1241x376 0.406 / 0.404 / 0.434 / 0.437 /
                    // 0.453 ms vs 0.357, 1280x720 0.90-1.17 vs 0.765
#endif
#if ORB_TU_MAIN
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KR_WAVES))) k_rerun(const uint8_t* __restrict__ pyr, uint32_t* __restrict__ cand,
                                               int* __restrict__ cellCount, Geom g,
                                               const CellGeom* __restrict__ cells, int NWG) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int b = blockIdx.x / NWG, gw = blockIdx.x - b * NWG, l = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const LevelGeom& lg = g.lv[l];
    const int nC = lg.rows * lg.cols;
    const CellGeom* lc = cells + lg.cell0;
    uint32_t* fcand = cand + (long long)b * g.candPerFrame;
    int* fcount = cellCount + (long long)b * g.nCells + lg.cell0;
    int ord = 0;
    for (int c0 = 0; c0 < nC; c0 += 64) {
        const int c = c0 + lane;
        bool fb = false;
        if (c < nC) {
            const CellGeom& cg = lc[c];
            const int cnt = fcount[c];
            const int n = (cg.hx <= 6 || cg.hy <= 6) ? 0 : min(cnt & COUNT_MASK, cg.cap);
            fb = (cnt & RERUN_FLAG) || (!cg.skipped && n <= 3);
        }
        uint64_t m = __ballot(fb);
        while (m) {
            const int cc = c0 + __builtin_ctzll(m);
            m &= m - 1;
            if (ord++ % NWG != gw) continue;
            const CellGeom cg = lc[cc];
            const int dw = cg.hx - 6, dh = cg.hy - 6;
            int n = 0;
            if (dw > 0 && dh > 0) {
                const uint8_t* det = pyr + lg.base + (long long)b * lg.fstride +
                                     (long long)(EDGE + cg.y0 + 3) * lg.pitch + EDGE + cg.x0 + 3;
                n = cell_fast_rerun(det, lg.pitch, dw, dh, cg.x0 + 3, cg.y0 + 3, 7, smem, fcand + cg.candOff, tid, l);
            }
            if (tid == 0) fcount[cc] = n | RERUN_FLAG;
        }
    }
}
#endif  // ORB_TU_MAIN

// ---- selection (retainBest replay) -------------------------------------------------------
struct ScoreGreater {  // KeypointResponseGreater on the packed FAST score
    ORB_HD bool operator()(uint32_t a, uint32_t b) const { return (a >> 24) > (b >> 24); }
};

// One workgroup per (level, frame).  In: each cell's NMS survivors at fastTh from k_fast, in
// arrival order, and their count.  (1) cells with <= 3 survivors are re-run at t = 7 (RERUN;
// otherwise k_rerun did it); (2) each
// cell's survivors are put in raster order — the order cv::FAST returns them, which
// retainBest's nth_element depends on; (3) nToRetain / redistribution (ORBextractor.cc:622-670);
// (4) retainBest per cell, concatenation in cell order, retainBest to the level quota
// (ORBextractor.cc:680-701) — exact libstdc++ nth_element replays.  Lists live in LDS when the
// level's survivors fit (Geom::selCap), otherwise in the frame's scratch area `cand2`.
#ifndef SELECT_CAP
#define SELECT_CAP 0  // > 0: survivors per level held in LDS for every geometry (experiments)
#endif
// survivors per level held in LDS (beyond: the global-scratch path, same result), per frame
// size: (W*H / 200) rounded down to 512 in [1024, 3072] -- 1536 at 640x480 (6 -> 10 work-groups
// per CU: 0.177 -> 0.146 ms with 3072), 2048 at 1241x376 (0.499 -> 0.474), 3072 at 1280x720
// (2048 there: 0.84 -> 1.14, most levels past LDS)
inline int select_cap(int w, int h) {
    if (SELECT_CAP > 0) return SELECT_CAP;
    return std::min(3072, std::max(1024, (int)(((long long)w * h / 200) & ~511ll)));
}
// KeypointResponseGreater on HARRIS_SCORE elements: float response in the high word, the
// packed FAST record (identity) in the low word.
struct HarrisGreater {
    __device__ bool operator()(uint64_t a, uint64_t b) const {
        return __uint_as_float((uint32_t)(a >> 32)) > __uint_as_float((uint32_t)(b >> 32));
    }
};

// HarrisResponses (ORBextractor.cc:79-120) at level pixel (x, y), blockSize 7, k = 0.04:
// cellImage is a view into the level, so the 7x7 block starts at (x-3, y-3) of the level.
// g++ -O3 -march=native contracts the response to fma(-(k*s), s, fma(A, B, -(C*C))) (oracle
// harris_responses, DESIGN.md §FP policy).
__device__ __forceinline__ float harris_response(const uint8_t* roi, int pitch, int x, int y, float scale4) {
    const uint8_t* p0 = roi + (long long)(y - 3) * pitch + (x - 3);
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const uint8_t* ptr = p0 + (long long)i * pitch + j;
            const int Ix = (ptr[1] - ptr[-1]) * 2 + (ptr[-pitch + 1] - ptr[-pitch - 1]) + (ptr[pitch + 1] - ptr[pitch - 1]);
            const int Iy = (ptr[pitch] - ptr[-pitch]) * 2 + (ptr[pitch - 1] - ptr[-pitch - 1]) + (ptr[pitch + 1] - ptr[-pitch + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    const float fa = (float)a, fb = (float)b, fc = (float)c;
    const float s = fa + fb;
    const float t3 = 0.04f * s;
    const float u = __builtin_fmaf(fa, fb, -(fc * fc));
    const float rsp = __builtin_fmaf(-t3, s, u);
    return rsp * scale4;
}

// Exclusive prefix of src[0..n) into dst[0..n], total into dst[n], on one wave (n <= 256).
__device__ __forceinline__ void wave_prefix(int* dst, const int* src, int n, int lane) {
    int carry = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int c = c0 + lane;
        const int v = c < n ? src[c] : 0;
        const int incl = wave_incl_scan(v);
        if (c < n) dst[c] = carry + incl - v;
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) dst[n] = carry;
}

__device__ __forceinline__ int wave_sum(int v) { return wave_total(v); }

// Cell of list element i: the last c in [0, n) with off[c] <= i (off ascending, off[0] = 0).
__device__ __forceinline__ int cell_of(const int* off, int n, int i) {
    int lo = 0, hi = n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

#ifndef KR_TAIL_BATCH
#define KR_TAIL_BATCH 256  // batches below this resize every level with its own launch
#endif
#ifndef KS_SEP_BATCH
#define KS_SEP_BATCH 32  // batches below this re-run FAST(7) cells in k_rerun, not in k_select
#endif
#ifndef KS_CELL_SPREAD
#define KS_CELL_SPREAD 1
#endif
#ifndef KS_SEP_PIXELS
#define KS_SEP_PIXELS 0  // and frames larger than this (0: every batch; the in-k_select re-run
                         // path stays for experiments: -DKS_SEP_PIXELS=100000000)
#endif
#ifndef KS_WAVES
#define KS_WAVES 2  // waves per SIMD the register allocation targets
#endif

// The last of a frame's L k_select workgroups to finish writes the frame's per-level (first output
// slot, count) pairs and total (what k_lvl_prefix did in a launch of its own): each workgroup's
// thread 0 publishes its level count with an agent-scope atomic store (past its XCD's L2: the
// frame's workgroups run on different XCDs), waits for it, then counts itself in selDone[b];
// the one that brings it to L reads the L counts with agent-scope atomic loads and resets
// selDone[b] for the next launch.  Ordering: the only data handed over (lvlCount) is written and
// read with agent-scope atomics, which bypass the XCD's L2, and the writer waits for its store to
// complete (vmcnt(0)) before it counts itself; the last workgroup then takes an agent-scope
// acquire (one L1 / L2 invalidate, on that workgroup only) before its loads.  (A __threadfence()
// release on every workgroup writes back the L2 of each: +60 us per c3 step.)
__device__ __forceinline__ void select_frame_done(int b, int L, int l, int keep, int* __restrict__ lvlCount,
                                                  int* __restrict__ selDone, int2* __restrict__ lvlInfo,
                                                  int* __restrict__ counts) {
    __hip_atomic_store(&lvlCount[(long long)b * L + l], keep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(&selDone[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != L - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    int c[ORB_MAX_LEVELS];
#pragma unroll
    for (int l = 0; l < ORB_MAX_LEVELS; ++l)
        c[l] = __hip_atomic_load(&lvlCount[(long long)b * L + min(l, L - 1)], __ATOMIC_RELAXED,  // (in bounds:
                                 __HIP_MEMORY_SCOPE_AGENT);                                      // all issued at once)
    int before = 0;
#pragma unroll
    for (int l = 0; l < ORB_MAX_LEVELS; ++l)
        if (l < L) {
            lvlInfo[(long long)b * ORB_MAX_LEVELS + l] = make_int2(before, c[l]);
            before += c[l];
        }
    counts[b] = before;
    __hip_atomic_store(&selDone[b], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#if ORB_TU_MAIN
template <bool HARRIS, bool RERUN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KS_WAVES))) k_select(const uint8_t* __restrict__ pyr, uint32_t* __restrict__ cand,
                                                uint32_t* __restrict__ cand2, int* __restrict__ cellCount, Geom g,
                                                const CellGeom* __restrict__ cells, uint32_t* __restrict__ lvlOut,
                                                int* __restrict__ lvlCount, uint64_t* __restrict__ candH,
                                                float* __restrict__ lvlResp, float harrisScale4, int* __restrict__ selDone,
                                                int2* __restrict__ lvlInfo, int* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_cnt[ORB_MAX_CELLS_PER_LEVEL];
    __shared__ int s_ret[ORB_MAX_CELLS_PER_LEVEL];
    __shared__ int s_off[ORB_MAX_CELLS_PER_LEVEL + 1];
    __shared__ int s_koff[ORB_MAX_CELLS_PER_LEVEL + 1];
    __shared__ uint8_t s_skip[ORB_MAX_CELLS_PER_LEVEL];
    __shared__ int s_fb[ORB_MAX_CELLS_PER_LEVEL + 1];  // cells to re-run at t = 7, count last
    __shared__ int s_coff[ORB_MAX_CELLS_PER_LEVEL];    // candOff of every cell
    // grid (frame, level): workgroup i runs on XCD i % 8, so every XCD gets every level (with
    // (level, frame) all the heavy level-0 lists landed on one XCD), heaviest level first
    const int b = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    KS_T(0);
    const LevelGeom& lg = g.lv[l];
    const int nC = lg.rows * lg.cols;
    const CellGeom* lc = cells + lg.cell0;
    uint32_t* fcand = cand + (long long)b * g.candPerFrame;
    int* fcount = cellCount + (long long)b * g.nCells + lg.cell0;
    if (wave == 0) {  // counts, skip flags, and the list of cells to re-run (ascending, RERUN)
        constexpr int CPL = ORB_MAX_CELLS_PER_LEVEL / 64;
        int cnt[CPL], cap[CPL], skip[CPL], hx[CPL], hy[CPL], coff[CPL];
#pragma unroll
        for (int j = 0; j < CPL; ++j) {  // every load of the wave in flight at once
            const int c = 64 * j + lane;
            if (c < nC) {
                cnt[j] = fcount[c];
                cap[j] = lc[c].cap;
                skip[j] = lc[c].skipped;
                hx[j] = lc[c].hx;
                hy[j] = lc[c].hy;
                coff[j] = lc[c].candOff;
            }
        }
        int nfb = 0;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = 64 * j + lane;
            bool fb = false;
            if (c < nC) {
                // (k_rerun's counts carry RERUN_FLAG; such a cell has been re-run: not again)
                const int n = (skip[j] || hx[j] <= 6 || hy[j] <= 6) ? 0 : min(cnt[j] & COUNT_MASK, cap[j]);
                s_cnt[c] = n;
                s_skip[c] = (uint8_t)skip[j];
                s_coff[c] = coff[j];
                fb = RERUN && !skip[j] && n <= 3;
            }
            const uint64_t m = __ballot(fb);
            if (fb) s_fb[nfb + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = c;
            nfb += __popcll(m);
        }
        if (lane == 0) s_fb[ORB_MAX_CELLS_PER_LEVEL] = nfb;
    }
    __syncthreads();
    // (1) FAST(cellImage, keys, 7, true) where a cell kept <= 3 (a skipped cell is `continue`d)
    {
        const int nfb = s_fb[ORB_MAX_CELLS_PER_LEVEL];
        for (int f = 0; f < (RERUN ? nfb : 0); ++f) {
            const int c = s_fb[f];
            const CellGeom cg = lc[c];
            const int dw = cg.hx - 6, dh = cg.hy - 6;
            int n = 0;
            if (dw > 0 && dh > 0) {
                const uint8_t* det = pyr + lg.base + (long long)b * lg.fstride +
                                     (long long)(EDGE + cg.y0 + 3) * lg.pitch + EDGE + cg.x0 + 3;
                n = cell_fast_rerun(det, lg.pitch, dw, dh, cg.x0 + 3, cg.y0 + 3, 7, smem, fcand + cg.candOff, tid, l);
            }
            if (tid == 0) {
                s_cnt[c] = n;
                fcount[c] = n;
            }
            __syncthreads();
        }
    }
    KS_T(1);
    if (wave == 0) {
        wave_prefix(s_off, s_cnt, nC, lane);
        // (3) nToRetain / nToDistribute / bNoMore bookkeeping (ORBextractor.cc:622-670), one
        // lane per cell: within a pass every cell's update reads only the pass constants, and
        // the pass totals are integer sums, so the lanes reproduce the sequential loop exactly.
        // A skipped cell keeps 0 and is not bNoMore after the first pass (the reference
        // `continue`s past it), then takes the tot = 0 branch of the redistribution.
        constexpr int CPL = ORB_MAX_CELLS_PER_LEVEL / 64;
        const int nfc = lg.nfc;
        int ret[CPL], tot[CPL];
        bool more[CPL];  // live and not bNoMore
        int dist = 0, nm = 0;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = 64 * j + lane;
            more[j] = false;
            ret[j] = 0;
            tot[j] = 0;
            if (c < nC) {
                const bool sk = s_skip[c] != 0;
                tot[j] = sk ? 0 : s_cnt[c];
                if (sk) {
                    more[j] = true;
                } else if (tot[j] > nfc) {
                    ret[j] = nfc;
                    more[j] = true;
                } else {
                    ret[j] = tot[j];
                    dist += nfc - tot[j];
                    nm++;
                }
            }
        }
        int nToDistribute = wave_sum(dist), nNoMore = wave_sum(nm);
        while (nToDistribute > 0 && nNoMore < nC) {
            const int nNew = nfc + (int)ceilf((float)nToDistribute / (nC - nNoMore));
            dist = 0;
            nm = 0;
#pragma unroll
            for (int j = 0; j < CPL; ++j) {
                if (!more[j]) continue;
                if (tot[j] > nNew) {
                    ret[j] = nNew;
                } else {
                    ret[j] = tot[j];
                    dist += nNew - tot[j];
                    more[j] = false;
                    nm++;
                }
            }
            nToDistribute = wave_sum(dist);
            nNoMore += wave_sum(nm);
        }
#pragma unroll
        for (int j = 0; j < CPL; ++j)
            if (64 * j + lane < nC) s_ret[64 * j + lane] = ret[j];
    }
    __syncthreads();
    KS_T(2);
    const int M = s_off[nC];
    const int selCap = g.selCap;
    const bool inLds = M <= selCap;
    uint32_t* raw = (uint32_t*)smem;                                      // arrival order
    uint32_t* srt = inLds ? raw + selCap : cand2 + (long long)b * g.candPerFrame;  // raster order
    const uint32_t* srcOf = inLds ? raw : fcand;
    if (inLds) {  // the level's survivors, cell after cell, one element per thread (4 loads in flight)
        for (int i0 = tid; i0 < M; i0 += 1024) {
            uint32_t v[4];
            int dsti[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + 256 * u;
                dsti[u] = -1;
                if (i < M) {
                    const int c = cell_of(s_off, nC, i);
                    v[u] = fcand[s_coff[c] + (i - s_off[c])];
                    dsti[u] = i;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (dsti[u] >= 0) raw[dsti[u]] = v[u];
        }
        __syncthreads();
        // (2) rank sort of each cell by position (positions are unique), one element per thread
        for (int i = tid; i < M; i += 256) {
            const int c = cell_of(s_off, nC, i);
            const int o = s_off[c], n = s_cnt[c];
            const uint32_t e = raw[i], key = e & 0xFFFFFFu;
            int r = 0;
            for (int j2 = 0; j2 < n; ++j2) r += (raw[o + j2] & 0xFFFFFFu) < key;
            srt[o + r] = e;
        }
    } else {
        // (2) as above on the frame's scratch area, one wave per cell
        for (int c = wave; c < nC; c += 4) {
            const int n = s_cnt[c];
            const uint32_t* seg = srcOf + lc[c].candOff;
            uint32_t* dst = srt + lc[c].candOff;
            for (int i = lane; i < n; i += 64) {
                const uint32_t e = seg[i], key = e & 0xFFFFFFu;
                int r = 0;
                for (int j2 = 0; j2 < n; ++j2) r += (seg[j2] & 0xFFFFFFu) < key;
                dst[r] = e;
            }
        }
    }
    __syncthreads();
    if constexpr (HARRIS) {
        // HarrisResponses on every cell keypoint (ORBextractor.cc:616-620), then the same
        // retention on (response, record) pairs
        uint64_t* hs = inLds ? (uint64_t*)(smem + (size_t)8 * selCap) : candH + (long long)b * g.candPerFrame;
        const uint8_t* roi = pyr + lg.base + (long long)b * lg.fstride + (long long)EDGE * lg.pitch + EDGE;
        for (int c = wave; c < nC; c += 4) {
            const int o = inLds ? s_off[c] : lc[c].candOff;
            for (int i = lane; i < s_cnt[c]; i += 64) {
                const uint32_t e = srt[o + i];
                const float r = harris_response(roi, lg.pitch, e & 0xFFF, (e >> 12) & 0xFFF, harrisScale4);
                hs[o + i] = ((uint64_t)__float_as_uint(r) << 32) | e;
            }
        }
        __syncthreads();
        HarrisGreater hcomp;
        for (int c = KS_CELL_SPREAD ? lane * 4 + wave : tid; c < nC; c += 256) {  // cell c on wave c % 4
            uint64_t* seg = hs + (inLds ? s_off[c] : lc[c].candOff);
            s_cnt[c] = orbsel::retain_best(seg, s_cnt[c], s_ret[c], hcomp);
        }
        __syncthreads();
        if (wave == 0) wave_prefix(s_koff, s_cnt, nC, lane);
        __syncthreads();
        const int K = s_koff[nC];
        uint64_t* list;
        if (inLds) {  // kept prefixes of hs -> the raw + srt region (disjoint)
            list = (uint64_t*)smem;
            for (int c = wave; c < nC; c += 4)
                for (int k = lane; k < s_cnt[c]; k += 64) list[s_koff[c] + k] = hs[s_off[c] + k];
        } else {
            list = hs + lc[0].candOff;
            if (tid == 0)
                for (int c = 0; c < nC; ++c) {
                    const uint64_t* src = hs + lc[c].candOff;
                    for (int k = 0; k < s_cnt[c]; ++k) list[s_koff[c] + k] = src[k];
                }
        }
        __syncthreads();
        int keep = K;
        if (K > lg.nDesired) {
            keep = lg.nDesired;
            if (tid == 0) orbsel::retain_best(list, K, lg.nDesired, hcomp);
        }
        __syncthreads();
        const long long ob = (long long)b * g.kpCap + lg.kpBase;
        for (int k = tid; k < keep; k += 256) {
            const uint64_t v = list[k];
            lvlOut[ob + k] = (uint32_t)v;
            lvlResp[ob + k] = __uint_as_float((uint32_t)(v >> 32));
        }
        if (tid == 0) {
            select_frame_done(b, g.L, l, keep, lvlCount, selDone, lvlInfo, counts);
        }
        return;
    }
    // (4) retainBest per cell, then the level list in cell order, then retainBest to the quota
    KS_T(3);
    ScoreGreater comp;
    // cells dealt round-robin over the four waves (cell c on wave c % 4): a level's few dozen
    // serial replays run on four SIMDs instead of one wave's lanes
    // (measured and dropped, round 4: cells of > 32 / 64 / 128 survivors retained by a whole wave
    // with the ballot partitions: k_select 71 -> 83-88 us c3, 105 -> 113-122 us c4)
    for (int c = KS_CELL_SPREAD ? lane * 4 + wave : tid; c < nC; c += 256) {
        uint32_t* seg = srt + (inLds ? s_off[c] : lc[c].candOff);
        s_cnt[c] = orbsel::retain_best(seg, s_cnt[c], s_ret[c], comp);
    }
    __syncthreads();
    KS_T(4);
    if (wave == 0) wave_prefix(s_koff, s_cnt, nC, lane);
    __syncthreads();
    const int K = s_koff[nC];
    uint32_t* list;
    if (inLds) {  // kept prefixes of srt -> raw (disjoint regions), one element per thread
        for (int i = tid; i < K; i += 256) {
            const int c = cell_of(s_koff, nC, i);
            raw[i] = srt[s_off[c] + (i - s_koff[c])];
        }
        list = raw;
    } else {  // sequential in-place compaction (dest <= src, ascending) in cand2's level area
        list = srt + lc[0].candOff;
        if (tid == 0)
            for (int c = 0; c < nC; ++c) {
                const uint32_t* src = srt + lc[c].candOff;
                for (int k = 0; k < s_cnt[c]; ++k) list[s_koff[c] + k] = src[k];
            }
    }
    __syncthreads();
    int keep = K;
    if (K > lg.nDesired) {
        keep = lg.nDesired;
        if (inLds) {  // one wave, partitions by ballot (nth_select.h); scratch = the free srt region
            uint16_t* Lp = (uint16_t*)srt;
            if (wave == 0)
                orbsel::retain_best_wave(list, K, lg.nDesired, comp, Lp, Lp + K, lane);
        } else if (tid == 0) {
            orbsel::retain_best(list, K, lg.nDesired, comp);
        }
    }
    __syncthreads();
    KS_T(5);
    uint32_t* out = lvlOut + (long long)b * g.kpCap + lg.kpBase;
    for (int k = tid; k < keep; k += 256) out[k] = list[k];
    if (tid == 0) {
        select_frame_done(b, g.L, l, keep, lvlCount, selDone, lvlInfo, counts);
    }
#if KS_TIMING
    // phases: 0 counts + re-runs, 1 bookkeeping, 2 load + raster sort, 3 per-cell retainBest,
    // 4 level list + level retainBest, 5 output; [6] = survivors M, [7] = workgroups
    if (tid == 0) {
        atomicAdd(&g_kstime[l][0], kst1 - kst0);
        atomicAdd(&g_kstime[l][1], kst2 - kst1);
        atomicAdd(&g_kstime[l][2], kst3 - kst2);
        atomicAdd(&g_kstime[l][3], kst4 - kst3);
        atomicAdd(&g_kstime[l][4], kst5 - kst4);
        atomicAdd(&g_kstime[l][5], __builtin_amdgcn_s_memrealtime() - kst5);
        atomicAdd(&g_kstime[l][6], (unsigned long long)M);
        atomicAdd(&g_kstime[l][7], 1ull);
    }
#endif
}
#endif  // ORB_TU_MAIN

// ---- FAST on the levels: per-tile detection + the per-cell non-max suppression --------------
// ComputeKeyPoints runs cv::FAST(cellImage, keys, fastTh, true) on every cell ROI of every
// level (ORBextractor.cc:560-607).  A cell's FAST sees its ROI only: detection rows / cols
// [3, n-3) of the ROI = the cell's detection area, and NMS neighbours outside that area count
// as 0.  Corner-ness and score are properties of the pixel alone, so one pass
// over each level's detection region [16, detX1) x [16, detY1) (the union of the cells'
// areas) finds every cell's corners; the NMS then applies each cell's own boundary.
//
// k_fast: one 256-thread workgroup per detection tile of a level, per frame.  A tile is tw4
// dwords (TW = 4 tw4 <= 256 columns, x0 a multiple of 4) by th rows: the level's detection width
// is split evenly into ceil(width / 256) tiles, so few lanes fall outside the region, and th is
// sized so the staged tile and the strength plane fit their LDS budgets.  The tile with its 1-px
// strength ring is one flattened (plane row, dword) index space of (th + 2) x (tw4 + 2) dwords
// (ring rows -1 and th; ring dwords -1 and tw4 contribute their one adjacent pixel), dealt to
// the 4 waves 64 dwords at a time:
//   (1) stage rows y0-4 .. y0+th+3, columns from the 16-aligned column at or below x0-8 to
//       x0+TW+7, into LDS with 16-byte loads, all in flight before any LDS write;
//   (2) compass pre-filter of cv::FAST (a 9-arc always covers two cyclically adjacent points of
//       {0, 4, 8, 12}) on the lane's 4 pixels, packed 16-bit; dwords with a survivor inside the
//       level's detection region are queued per wave;
//   (3) the queue: expanded to one pixel per slot, the exact strength S (score = S - 1) in full
//       64-pixel passes, `S > fastTh ? S : 0` into an LDS strength plane (a pixel the compass
//       rejects is no corner at fastTh and keeps 0: the NMS only reads S > fastTh);
//   (4) after one barrier, the plane's interior corners (flattened again) and the per-cell 3x3
//       strict NMS; survivors are appended to their cell's candidate slots as
//       ((S-1) << 24) | (y << 12) | x (k_select restores raster order).
// The 7x7 blur of the descriptors is not materialised: k_orient_desc evaluates it at the
// rBRIEF sample points from a raw window (ORBextractor.cc:760).
#define FT_TW_MAX 256     // detection columns per tile at most (64 lanes x 4 pixels)
#define FT_IN_BYTES 12672  // staged-tile LDS budget (44 rows of 288 B at TW = 256)
#define FT_S_BYTES 10032   // strength-plane LDS budget (38 rows of 264 B at TW = 256; a multiple of 16)
static_assert(FT_S_BYTES % 16 == 0 && FT_IN_BYTES % 16 == 0, "k_fast's LDS buffers are cleared / staged in 16-B units");
#define FT_Q 512           // per-wave queue (u16 entries): dwords, then the NMS corner list
#define FT_CQ 320          // per-wave pixel list (u16 entries): < 64 carried + 256 expanded
#define FT_CL 256          // per-wave corner list (u16 entries) filled by the strength passes; a
                           // workgroup where a wave has more corners scans the strength plane instead
                           // (Geom::fastCl lowers the cap for the fallback's parity test)
struct FastTile {
    int level, x0, y0;  // detection origin (level coordinates); x0 = 16 + k TW, a multiple of 4
    int tw4, th;        // dwords per row (>= 2), rows (clipped to the detection region)
    int sp, sx;         // staged row pitch (bytes, a multiple of 16); x0 - first staged column (8 .. 23)
    uint32_t rcpF;      // ceil(2^32 / (tw4 + 2)): flattened ring index -> plane row
    uint32_t rcpI;      // ceil(2^32 / tw4): interior index -> row
    uint32_t rcpU;      // ceil(2^32 / (sp / 16)): staged unit -> row
};

#ifndef KF_DPL
#define KF_DPL 2  // adjacent dwords per lane and step of the compass loop (1, 2 or 4)
#endif
#ifndef KF_B64
#define KF_B64 1  // compass groups on 8-B aligned dword pairs read with ds_read_b64 (KF_DPL 2 only)
#endif
#if KF_B64
static_assert(KF_DPL == 2, "KF_B64 reads the groups' dword pairs");
#endif
#if ORB_ILP_HERE
__global__ void __launch_bounds__(256) k_fast(const uint8_t* __restrict__ pyr, Geom g,
                                                      const FastTile* __restrict__ tiles,
                                                      uint32_t* __restrict__ cand, int* __restrict__ cellCount) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[FT_IN_BYTES];
    __shared__ __attribute__((aligned(16))) uint8_t s_S[FT_S_BYTES];
    // per-wave lists; the last slot of each is a trash slot, so ballot-compacted appends store
    // unconditionally (no exec-mask branch per append)
    __shared__ uint16_t s_q[4][FT_Q + 2];
    __shared__ uint16_t s_px[4][FT_CQ + 2];  // a chunk's pixels, compacted in place to its corners
    __shared__ uint16_t s_cl[4][FT_CL + 2];  // the wave's interior corners (tile row << 9 | tile column)
    __shared__ int s_ovf;                    // a wave's corner list overflowed: scan the plane
    __shared__ uint8_t s_cm[FT_TW_MAX / 4 + 3 + KF_DPL];  // per flattened dword column: its detection
                                                           // pixels (0 past the ring; KF_B64: index
                                                           // dc + 1, 0 at dc = -1)
    KF_T(0);
    // (plain block order: an XCD-aware order, vertically adjacent tiles on one XCD so their halo
    // rows hit in its L2, measured slower -- 0.646 vs 0.574 ms c3: the halo is not what binds)
    FastTile t = tiles[blockIdx.x];
    const int b = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // the level's geometry and the tile in SGPRs for the whole kernel (read through a reference
    // into the kernarg block, the compiler re-issued dependent s_loads inside the loops); the
    // empty asm makes the copies opaque, so they cannot be rematerialised
    LevelGeom lg = g.lv[t.level];
    asm volatile("" : "+s"(lg.w), "+s"(lg.h), "+s"(lg.pitch), "+s"(lg.ph), "+s"(lg.detX1), "+s"(lg.detY1),
                 "+s"(lg.rows), "+s"(lg.cols));
    asm volatile("" : "+s"(lg.cellW), "+s"(lg.cellH), "+s"(lg.cellWm), "+s"(lg.cellHm), "+s"(lg.cell0),
                 "+s"(lg.base), "+s"(lg.fstride), "+s"(lg.candBase), "+s"(lg.capMax));
    asm volatile("" : "+s"(t.x0), "+s"(t.y0), "+s"(t.tw4), "+s"(t.th), "+s"(t.sp), "+s"(t.sx), "+s"(t.rcpF),
                 "+s"(t.rcpI));
    const int fw = t.tw4 + 2;          // flattened row width (dwords): ring dword -1 .. tw4
    const int spw = 4 * t.tw4 + 8;     // strength-plane pitch: tile columns -4 .. TW+3
    {  // (1) stage: padded rows y0+12 .. (clipped to the buffer), t.sp bytes from the 16-aligned
       // padded column x0+16-sx (clipped to the row)
        const uint8_t* src = pyr + lg.base + (long long)b * lg.fstride;
        const int pr0 = t.y0 - 4 + EDGE, pc0 = t.x0 - t.sx + EDGE;
        const int upr = t.sp >> 4;
        const int rows = min(t.th + 8, lg.ph - pr0);
        const int units = min(upr, (lg.pitch - pc0) >> 4);
        const int nU = (t.th + 8) * upr;  // <= FT_IN_BYTES / 16
        const uint4* gs = (const uint4*)(src + (long long)pr0 * lg.pitch + pc0);
        const int gsu = lg.pitch >> 4;
        constexpr int NU = (FT_IN_BYTES / 16 + 255) / 256;
        uint4 v[NU];
#pragma unroll
        for (int k = 0; k < NU; ++k) {
            const int i = tid + 256 * k;
            const int r = (int)__umulhi((uint32_t)i, t.rcpU), u = i - r * upr;
            const bool ok = i < nU && r < rows && u < units;
            v[k] = gs[ok ? (long long)r * gsu + u : 0ll];  // every slot loads (no scratch spill)
            if (!ok) v[k] = make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < NU; ++k) {
            const int i = tid + 256 * k;
            if (i < nU) ((uint4*)s_in)[i] = v[k];
        }
        // the strength plane zeroed with 16-B stores (FT_S_BYTES is a multiple of 16)
        const int nS = ((t.th + 2) * spw + 15) >> 4;
        for (int i = tid; i < nS; i += 256) ((uint4*)s_S)[i] = make_uint4(0u, 0u, 0u, 0u);
        if (tid == 0) s_ovf = 0;
#if KF_B64
        if (tid < fw + 3) {
            const int dc = tid - 1, X = t.x0 + 4 * (dc - 1);
            const int lo = max(dc == 0 ? 3 : 0, EDGE - X), hi = min(dc == fw - 1 ? 1 : 4, lg.detX1 - X);
            s_cm[tid] = (uint8_t)(dc >= 0 && dc < fw && lo < hi ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u);
        }
#else
        if (tid < fw) {
            // dword column dc: pixels X .. X + 3, X = x0 + 4 (dc - 1); the ring columns contribute
            // the one pixel next to the tile, every pixel inside the detection region [16, detX1)
            const int dc = tid, X = t.x0 + 4 * (dc - 1);
            const int lo = max(dc == 0 ? 3 : 0, EDGE - X), hi = min(dc == fw - 1 ? 1 : 4, lg.detX1 - X);
            s_cm[dc] = (uint8_t)(lo < hi ? (((1u << hi) - 1u) & ~((1u << lo) - 1u)) : 0u);
        }
        if (tid >= fw && tid < fw + KF_DPL) s_cm[tid] = 0;  // the compass groups' dwords past the ring
#endif
    }
    __syncthreads();
    KF_T(1);
    const int ft = g.fastTh;
    const uint32_t tt = (uint32_t)ft | ((uint32_t)ft << 16);
    uint16_t* pq = s_q[wave];
    uint16_t* px = s_px[wave];
    // pixel code = plane row << 9 | plane column (plane row = tile row + 1, plane column = tile
    // column + 1); staged byte of a pixel: row pr + 3, column sx + pc - 1
    int np = 0;
    int ncl = 0;  // the wave's corners so far (wave-uniform)
    uint16_t* cl = s_cl[wave];
    auto strength_pass = [&](int base, int n) {  // px[base .. base + n), n <= 64
        bool corner = false;
        uint16_t code = 0;
        if (lane < n) {
            const uint16_t c = px[base + lane];
            const int S = fast_strength_packed(s_in + ((c >> 9) + 3) * t.sp + t.sx + (c & 511) - 1, t.sp);
            s_S[(c >> 9) * spw + (c & 511) + 3] = (uint8_t)(S > ft ? S : 0);  // each pixel once
            // an NMS candidate: a corner inside the tile (plane rows 1 .. th, columns 1 .. TW)
            const int pr = c >> 9, pc = c & 511;
            corner = S > ft && pr >= 1 && pr <= t.th && pc >= 1 && pc <= 4 * t.tw4;
            code = (uint16_t)(((pr - 1) << 9) | (pc - 1));
        }
        const uint64_t m = __ballot(corner);
        if (corner) {
            const int ix = ncl + lanes_below(m);
            cl[ix < g.fastCl ? ix : FT_CL] = code;  // FT_CL: trash slot
        }
        ncl += __popcll(m);
    };
    // queue entry = flattened index f << 4 | mask (bit j: pixel j of dword f); f = pr * fw + dc,
    // dword dc - 1 of plane row pr, pixel j at plane column 4 dc + j - 3
    auto drain = [&](int qn) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int i0 = 0; i0 < qn; i0 += 64) {
            const int i = i0 + lane;
            const uint32_t e = i < qn ? pq[i] : 0u;
            const int f = (int)(e >> 4);
            const int pr = (int)__umulhi((uint32_t)f, t.rcpF), dc = f - pr * fw;
            const uint32_t code = ((uint32_t)pr << 9) + 4u * (uint32_t)dc - 3u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // expand the 64 entries into one pixel per slot
                const bool v = (e >> j) & 1u;
                const uint64_t m = __ballot(v);
                // every lane computes its slot, and the ballot itself selects it (one compare per bit)
                px[select_by_mask(m, FT_CQ, np + lanes_below(m))] = (uint16_t)(code + j);
                np += __popcll(m);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // full passes from the top of the list (the next expansion overwrites what they read:
            // LDS accesses of one wave complete in issue order)
            while (np >= 64) {
                np -= 64;
                strength_pass(np, 64);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    // (2) compass pre-filter over the flattened tile + ring, 64 dwords per wave and step
#if KF_TIMING
    unsigned long long kft2 = 0;
#endif
    {
        // KF_DPL adjacent dwords (4 KF_DPL pixels) per lane and step: a group shares its left /
        // centre / right loads and the step bookkeeping (one dword per lane before: 484 -> 466 us
        // per 512 c3 frames with two, 700 -> 669 c4, 9.52 -> 8.95 ms per 4096 720p).  Group
        // index g = pr * fwg + k over the plane rows whose level row lies in the detection region
        // (only the two ring rows can fall outside, so the region test is the loop's row range);
        // group k covers dwords KF_DPL k .. KF_DPL k + KF_DPL - 1 (those past the ring, fw ..,
        // have no detection pixel: s_cm is 0 there)
        int qn = 0;
#if KF_B64
        // group kp = dwords dc = 2 kp - 1, 2 kp (kp = 0: dc = -1 is a dummy with no detection
        // pixel): with the tile's first staged byte sx = 16 or 24 (host: tile widths a multiple of
        // 8 columns) every group's pair is 8-B aligned, so its row (and the left / right
        // neighbours, up and down rows) are five ds_read_b64: a wave's 32-lane half reads 64
        // consecutive dwords, conflict-free (the dword reads at an 8-B lane stride were 2-way
        // bank conflicts: dword banks are (a / 4) mod 32, 64-bit reads' (a / 4) mod 64)
        const int iw2 = t.sp >> 3, fwg = (fw >> 1) + 1;
#else
        const int iw = t.sp >> 2, fwg = (fw + KF_DPL - 1) / KF_DPL;
#endif
        const int prLo = max(0, EDGE + 1 - t.y0), prHi = min(t.th + 2, lg.detY1 + 1 - t.y0);  // wave-uniform
        const int nP = (prHi - prLo) * fwg;
        const int q256 = 256 / fwg, r256 = 256 - q256 * fwg;
        const int adStep = q256 * t.sp + 4 * KF_DPL * r256, adWrap = t.sp - 4 * KF_DPL * fwg;
        int g = wave * 64 + lane;
        int pr = g / fwg, kp = g - pr * fwg;
        pr += prLo;
#if KF_B64
        int ad = (pr + 3) * t.sp + t.sx + 8 * kp - 8;  // byte offset of the group's first dword (dc = 2 kp - 1)
        const int adSafe = 3 * t.sp + 16;
#else
        int ad = (pr + 3) * t.sp + t.sx + 4 * (KF_DPL * kp - 1);  // byte offset of the group's first dword
        const int adSafe = 3 * t.sp + 4;
#endif
        for (int it = wave; it * 64 < nP; it = __builtin_amdgcn_readfirstlane(it + 4)) {  // wave-uniform
            const bool valid = g < nP;
            uint32_t h[KF_DPL + 2];  // dwords -1 .. KF_DPL of the group's row
            uint32_t upv[KF_DPL], dnv[KF_DPL];
#if KF_B64
            const uint2* row2 = (const uint2*)(s_in + (valid ? ad : adSafe));
            {
                const uint2 L = row2[-1], C = row2[0], R = row2[1], U = row2[-3 * iw2], D = row2[3 * iw2];
                h[0] = L.y;
                h[1] = C.x;
                h[2] = C.y;
                h[3] = R.x;
                upv[0] = U.x;
                upv[1] = U.y;
                dnv[0] = D.x;
                dnv[1] = D.y;
            }
            const int dc = valid ? 2 * kp : fw + 1;  // s_cm index of the group's first dword (0 past the ring)
            const int fq = pr * fw + 2 * kp - 1;
#else
            const uint32_t* row = (const uint32_t*)(s_in + (valid ? ad : adSafe));
#pragma unroll
            for (int j = 0; j < KF_DPL + 2; ++j) h[j] = row[j - 1];
#pragma unroll
            for (int j = 0; j < KF_DPL; ++j) {
                upv[j] = row[j - 3 * iw];
                dnv[j] = row[j + 3 * iw];
            }
            const int dc = valid ? KF_DPL * kp : fw;  // s_cm[fw ..] = 0: nothing queued
            const int fq = pr * fw + KF_DPL * kp;
#endif
            // the row's dwords split once into even / odd byte lanes: a dword's q4 / q12 (pixels
            // x+3 / x-3) are the odd / even lanes of its neighbours, one v_alignbyte where they
            // straddle two dwords
            uint32_t he[KF_DPL + 2], ho[KF_DPL + 2];
#pragma unroll
            for (int j = 0; j < KF_DPL + 2; ++j) {
                he[j] = even_bytes(h[j]);
                ho[j] = odd_bytes(h[j]);
            }
            uint32_t m[KF_DPL];
#pragma unroll
            for (int j = 0; j < KF_DPL; ++j) {
                const uint32_t up = upv[j], dn = dnv[j];
                // even lanes (x, x+2): q4 = x+3, x+5 (odd bytes 3 / 1 of dwords 0 / +1), q12 = x-3, x-1
                const uint32_t pe = compass_half(he[j + 1], even_bytes(dn), __builtin_amdgcn_alignbyte(ho[j + 2], ho[j + 1], 2),
                                                 even_bytes(up), ho[j], tt);
                // odd lanes (x+1, x+3): q4 = x+4, x+6 (even bytes of +1), q12 = x-2, x (bytes 2 / 0 of -1 / 0)
                const uint32_t po = compass_half(ho[j + 1], odd_bytes(dn), he[j + 2], odd_bytes(up),
                                                 __builtin_amdgcn_alignbyte(he[j + 1], he[j], 2), tt);
                m[j] = compass_mask(pe, po) & s_cm[dc + j];
            }
            g += 256;
            kp += r256;
            pr += q256;
            ad += adStep;
            if (kp >= fwg) {
                kp -= fwg;
                pr += 1;
                ad += adWrap;
            }
            if (qn > FT_Q - 64 * KF_DPL) {
                drain(qn);
                qn = 0;
            }
#pragma unroll
            for (int j = 0; j < KF_DPL; ++j) {
                const bool v = m[j] != 0u;
                const uint64_t bm = __ballot(v);
                pq[select_by_mask(bm, FT_Q, qn + lanes_below(bm))] = (uint16_t)(((uint32_t)(fq + j) << 4) | m[j]);
                qn += (int)__popcll(bm);
            }
        }
#if KF_TIMING
        kft2 = __builtin_amdgcn_s_memrealtime();
#endif
        drain(qn);
        if (np) strength_pass(0, np);  // the remainder, < 64 pixels
    }
    if (ncl > g.fastCl && lane == 0) s_ovf = 1;
    KF_T(3);
    __syncthreads();
    KF_T(4);
    // (4) in-cell NMS.  Cell (i, j) has the detection area [16 + j*cellW, j == cols-1 ? w-16 :
    // 16 + (j+1)*cellW) in x (likewise in y), ORBextractor.cc:572-597; cell of a detection pixel:
    // ((y-16) / cellH, (x-16) / cellW) by exact reciprocal multiplies (host-checked).
    int* fcount = cellCount + (long long)b * g.nCells + lg.cell0;
    uint32_t* fcand = cand + (long long)b * g.candPerFrame + lg.candBase;
    // the tile's cells: rows ciT0 .. ciT1, columns cjT0 .. cjT0 + ncT - 1 (wave-uniform)
    const int ciT0 = (int)__umulhi((uint32_t)(t.y0 - EDGE), (uint32_t)lg.cellHm);
    const int ciT1 = (int)__umulhi((uint32_t)(t.y0 + t.th - 1 - EDGE), (uint32_t)lg.cellHm);
    const int cjT0 = (int)__umulhi((uint32_t)(t.x0 - EDGE), (uint32_t)lg.cellWm);
    const int cjT1 = (int)__umulhi((uint32_t)(min(t.x0 + 4 * t.tw4, lg.detX1) - 1 - EDGE), (uint32_t)lg.cellWm);
    const int ncT = cjT1 - cjT0 + 1, nT = (ciT1 - ciT0 + 1) * ncT;
    // KF_AGG: the survivors' cell slots taken per workgroup -- an LDS count per cell of the tile,
    // one global atomicAdd per cell, each survivor at the cell's base + its LDS rank -- instead of
    // one returning global atomic per survivor on the few counters of the tile's cells (their
    // same-address serialisation at L2 cost ~0.05 ms per c3 step: timing ablation `kf_noemit`,
    // profiles/r06/r06_w_summary.txt).  The counts and bases overlay s_px, the ranks s_in (both
    // free after the strength passes).
#ifndef KF_AGG
#define KF_AGG 1
#endif
    int* s_cc = (int*)s_px[0];
    int* s_base = s_cc + 64;
    uint16_t* s_rk = (uint16_t*)s_in;
    static_assert(sizeof(s_px) >= 128 * sizeof(int) && FT_IN_BYTES >= 4 * FT_CL * 2, "KF_AGG's LDS overlays");
    auto nms_emit = [&](const uint16_t* list, int n, auto aggC) {  // list == pq, or a list disjoint from it
        constexpr bool AGG = decltype(aggC)::value;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        int sn = 0;
        for (int k0 = 0; k0 < n; k0 += 64) {
            const int k = k0 + lane;
            bool keep = false;
            uint16_t e = 0;
            if (k < n) {
                e = list[k];
                const int rt = e >> 9, ct = e & 511;
                const int X = t.x0 + ct, Y = t.y0 + rt;
                const int ci = (int)__umulhi((uint32_t)(Y - EDGE), (uint32_t)lg.cellHm);
                const int cj = (int)__umulhi((uint32_t)(X - EDGE), (uint32_t)lg.cellWm);
                if (ci < lg.rows && cj < lg.cols) {
                    const int xlo = EDGE + cj * lg.cellW, xhi = cj == lg.cols - 1 ? lg.w - EDGE : xlo + lg.cellW;
                    const int ylo = EDGE + ci * lg.cellH, yhi = ci == lg.rows - 1 ? lg.h - EDGE : ylo + lg.cellH;
                    // the plane holds the tile's 1-px ring, so all 9 reads are in bounds: issue
                    // them together (no per-neighbour branch), then mask the out-of-cell ones
                    const uint8_t* sp = s_S + (rt + 1) * spw + ct + 4;
                    int nbv[9];
#pragma unroll
                    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                        for (int dx = -1; dx <= 1; ++dx) nbv[(dy + 1) * 3 + dx + 1] = sp[dy * spw + dx];
                    const int S = nbv[4];
                    const bool xl = X - 1 >= xlo, xr = X + 1 < xhi, yu = Y - 1 >= ylo, yd = Y + 1 < yhi;
                    bool ok = true;
#pragma unroll
                    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                        for (int dx = -1; dx <= 1; ++dx) {
                            if (dx == 0 && dy == 0) continue;
                            const bool inCell = (dx < 0 ? xl : dx > 0 ? xr : true) & (dy < 0 ? yu : dy > 0 ? yd : true);
                            const int nb = inCell ? nbv[(dy + 1) * 3 + dx + 1] : 0;
                            ok &= S - 1 > (nb ? nb - 1 : 0);
                        }
                    keep = ok;
                }
            }
            // survivors overwrite the front of the list (k0 + 64 > sn: no unread entry is hit)
            const uint64_t m = __ballot(keep);
            pq[select_by_mask(m, FT_Q, sn + lanes_below(m))] = e;
            sn += __popcll(m);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int k = lane; k < sn; k += 64) {
            const uint16_t e = pq[k];
            const int rt = e >> 9, ct = e & 511;
            const int X = t.x0 + ct, Y = t.y0 + rt;
            const int ci = (int)__umulhi((uint32_t)(Y - EDGE), (uint32_t)lg.cellHm);
            const int cj = (int)__umulhi((uint32_t)(X - EDGE), (uint32_t)lg.cellWm);
            if constexpr (AGG) {
                s_rk[wave * FT_CL + k] = (uint16_t)atomicAdd(&s_cc[(ci - ciT0) * ncT + (cj - cjT0)], 1);
            } else {
                const int c = ci * lg.cols + cj;
                const int S = s_S[(rt + 1) * spw + ct + 4];
                const int pos = atomicAdd(fcount + c, 1);
                if (pos < lg.capMax)
                    fcand[c * lg.capMax + pos] = ((uint32_t)(S - 1) << 24) | ((uint32_t)Y << 12) | (uint32_t)X;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        return sn;
    };
    // the NMS on the wave's own corner list (filled by its strength passes), or, where a wave's
    // list overflowed, on the plane's interior corners (ballot-compacted, flattened over th x
    // tw4 dwords) by all waves
    if (KF_AGG && !s_ovf && nT <= 64) {  // (workgroup-uniform)
        if (tid < 64) s_cc[tid] = 0;
        __syncthreads();
        const int sn = ncl ? nms_emit(cl, ncl, std::true_type{}) : 0;
        __syncthreads();
        if (tid < nT) {
            const int cnt = s_cc[tid];
            if (cnt) s_base[tid] = atomicAdd(fcount + (ciT0 + tid / ncT) * lg.cols + cjT0 + tid % ncT, cnt);
        }
        __syncthreads();
        for (int k = lane; k < sn; k += 64) {
            const uint16_t e = pq[k];
            const int rt = e >> 9, ct = e & 511;
            const int X = t.x0 + ct, Y = t.y0 + rt;
            const int ci = (int)__umulhi((uint32_t)(Y - EDGE), (uint32_t)lg.cellHm);
            const int cj = (int)__umulhi((uint32_t)(X - EDGE), (uint32_t)lg.cellWm);
            const int S = s_S[(rt + 1) * spw + ct + 4];
            const int pos = s_base[(ci - ciT0) * ncT + (cj - cjT0)] + s_rk[wave * FT_CL + k];
            if (pos < lg.capMax)
                fcand[(ci * lg.cols + cj) * lg.capMax + pos] = ((uint32_t)(S - 1) << 24) | ((uint32_t)Y << 12) | (uint32_t)X;
        }
    } else if (!s_ovf) {
        if (ncl) nms_emit(cl, ncl, std::false_type{});
    } else {
        int cn = 0;
        const int nI = t.th * t.tw4;
        for (int it = wave; it * 64 < nI; it += 4) {  // wave-uniform
            const int i = it * 64 + lane;
            uint32_t w4 = 0u;
            int r = 0, d = 0;
            if (i < nI) {
                r = (int)__umulhi((uint32_t)i, t.rcpI);
                d = i - r * t.tw4;
                w4 = *(const uint32_t*)(s_S + (r + 1) * spw + 4 + 4 * d);
            }
            if (__ballot(w4 != 0u) == 0ull) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool v = ((w4 >> (8 * j)) & 0xFFu) != 0u;
                const uint64_t m = __ballot(v);
                pq[select_by_mask(m, FT_Q, cn + lanes_below(m))] = (uint16_t)((r << 9) | (4 * d + j));
                cn += __popcll(m);
            }
            if (cn > FT_Q - 256) {
                nms_emit(pq, cn, std::false_type{});
                cn = 0;
            }
        }
        if (cn) nms_emit(pq, cn, std::false_type{});
    }
#if KF_TIMING
    KF_T(5);
    if (lane == 0) {
        atomicAdd(&g_kftime[0], kft1 - kft0);
        atomicAdd(&g_kftime[1], kft2 - kft1);
        atomicAdd(&g_kftime[2], kft3 - kft2);
        atomicAdd(&g_kftime[3], kft4 - kft3);
        atomicAdd(&g_kftime[4], kft5 - kft4);
        atomicAdd(&g_kftime[5], 1ull);
    }
#endif
}
#endif  // ORB_ILP_HERE

// ---- orientation + descriptor -------------------------------------------------------------
// One wave per keypoint slot.  Two memory round trips per wave: (1) the slot's packed record
// and the frame's per-level counts; (2) the raw 43x43 window around the keypoint (rows y-21 ..
// y+21, 16-byte loads into the wave's own LDS: 64 B per row from the 16-aligned column
// (x-5) & ~15 of the padded level).  From the window:
//   * IC_Angle (ORBextractor.cc:124-151) on its raw 31x31 disc;
//   * the descriptor image the reference reads after GaussianBlur(level ROI, 7x7, sigma 2)
//     in place (ORBextractor.cc:760), only where rBRIEF samples it: the row pass of the
//     fixed-point kernel (18, 34, 49, 55, 49, 34, 18) over the window's rows on the matrix
//     cores (three v_mfma_i32_16x16x64_i8 M-tiles x four N-tiles against a banded tap matrix),
//     stored as u16 sums in LDS, rows interleaved in pairs; then per sample the column pass by
//     four v_dot2 over row pairs, OpenCV's rounding for that column (SSE2 columns
//     x < 4*floor(w/4) half-to-even, the scalar tail half-up), or the raw
//     border byte where the sample lies outside the ROI (in-place ROI blur: the padding stays
//     un-blurred).  Exact integers throughout (T <= 257 * 65535 < 2^24).
// OD_WAVES keypoint slots per workgroup.  A wave's window and sums are its own (LDS is in order
// per wave); the two workgroup barriers only hand the IC moments to wave 0, which computes the
// slots' angle / sin / cos once, and hand those back.
#define OD_WR 21   // window reach: rBRIEF |offset| <= 18 + the blur's 3
#ifndef OD_WP
#define OD_WP 64   // LDS row pitch of the raw window (bytes).  80 (row blocks 4 rows apart on
                   // different banks: the row pass's 7-way conflicts become 2-way) measured
                   // slower: 640x480 0.607 vs 0.597 ms, 1241x376 1.183 vs 1.172
#endif
#define OD_HC 40   // row-pass columns: x-18 .. x+21 (10 groups of 4)
#define OD_HPR 22  // row pairs of the row-pass sums (window rows 0 .. 43)
#define OD_HN 56   // row-pass sum columns per pair row (window columns n = 0 .. 55 >= o0 + 39; hc = n - o0)
#define OD_BUF (OD_HPR * OD_HN * 4)  // per-wave LDS: the 44-row window, then (overlaid) the sums
static_assert(48 * OD_WP <= OD_BUF, "window rows 0 .. 47 inside the wave's buffer");
typedef int i32x4v __attribute__((ext_vector_type(4)));
// first window row of the three row-pass M-tiles (rows 28 .. 31 computed twice, identically)
__device__ constexpr int kOdRow[3] = {0, 16, 28};
// column-pass taps over row pairs (low half = the even row): rows r0-3 .. r0+4 when r0 is even
#define GP_E0 (18u | (34u << 16))
#define GP_E1 (49u | (55u << 16))
#define GP_E2 (49u | (34u << 16))
#define GP_E3 (18u | (0u << 16))
// ... and rows r0-4 .. r0+3 when r0 is odd (the even row of the first pair is r0-1, tap 0)
#define GP_O0 (0u | (18u << 16))
#define GP_O1 (34u | (49u << 16))
#define GP_O2 (55u | (49u << 16))
#define GP_O3 (34u | (18u << 16))

typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2u(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, a), __builtin_bit_cast(u16x2v, b), c, false);
}

// Column pass at window column hc (= dx + 18), sums of window rows r0 .. r0+6 (r0 = dy + 18):
// T = sum_j k_j H(r0 + 3 + j).  Row pairs p0 .. p0+3 hold rows 2 p0 .. 2 p0 + 7; for odd r0 the
// taps shift by one row (one u16 lane).
__device__ __forceinline__ uint32_t vpass(const uint32_t* __restrict__ Hs, int r0, int hc) {
    const int p0 = r0 >> 1;
    const uint32_t* q = Hs + p0 * OD_HN + hc;
    const uint32_t h0 = q[0], h1 = q[OD_HN], h2 = q[2 * OD_HN], h3 = q[3 * OD_HN];
    const bool odd = r0 & 1;
    const uint32_t t0 = odd ? GP_O0 : GP_E0, t1 = odd ? GP_O1 : GP_E1;
    const uint32_t t2 = odd ? GP_O2 : GP_E2, t3 = odd ? GP_O3 : GP_E3;
    return dot2u(h3, t3, dot2u(h2, t2, dot2u(h1, t1, dot2u(h0, t0, 0u))));
}


// cvRound-equivalent of T / 65536: half to even (SSE2 columns) or half up (scalar tail), then
// the saturating cast.
__device__ __forceinline__ uint32_t blur_round(uint32_t T, bool tail) {
    const uint32_t bias = tail ? 1u : ((T >> 16) & 1u);
    return min((T + 0x7FFFu + bias) >> 16, 255u);
}

#ifndef OD_SB
#define OD_SB 0  // 1: the shared-blur variant: both blur passes on the matrix cores
#endif
typedef _Float16 od_f16x8 __attribute__((ext_vector_type(8)));
typedef float od_f32x4 __attribute__((ext_vector_type(4)));
#define OD_SBP 14  // OD_SB: dwords per column of the blurred window (column-major; 14: conflict-free stores)
#ifndef OD_WAVES
#define OD_WAVES 4  // keypoint slots (waves) per workgroup (8 / 2 measured slower: 0.521 / 0.474 vs 0.468 ms c3;
                    // two slots per wave, lanes 0-31 / 32-63, 2 or 4 waves per workgroup: 0.531 / 0.567 vs
                    // 0.428 ms c3, 1.018 / 1.093 vs 0.818 c4 -- half the waves per CU, longer chains)
#endif
#if OD_SB
#define OD_ATTR __attribute__((amdgpu_waves_per_eu(8)))
#else
#define OD_ATTR
#endif
#if ORB_TU_MAIN
__global__ void __launch_bounds__(64 * OD_WAVES) OD_ATTR k_orient_desc(const uint8_t* __restrict__ pyr, Geom g,
                                                     const uint32_t* __restrict__ lvlOut,
                                                     const uint8_t* __restrict__ slotLvl,
                                                     const int2* __restrict__ lvlInfo, orb_keypoint_t* __restrict__ kps,
                                                     uint8_t* __restrict__ desc, const float* __restrict__ lvlResp) {
    // per wave: the raw window, then (overlaid) the row-pass sums
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[OD_WAVES][OD_BUF];
    __shared__ int2 s_mom[OD_WAVES];     // the waves' IC moments (m01, m10)
    __shared__ float4 s_trig[OD_WAVES];  // angle, sin, cos of the waves' keypoints
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // XCD-aware block order: workgroup i runs on XCD i % 8, so give each XCD a contiguous run
    // of keypoints (neighbouring keypoints share window rows: L2 hits instead of HBM re-reads)
    int bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int full = (gridDim.x * gridDim.y) & ~7;
    if (bid < full) bid = (bid & 7) * (full >> 3) + (bid >> 3);
    const int b = (int)__umulhi((uint32_t)bid, g.odDivMagic);  // bid / gridDim.x (exact: bid * gridDim.x < 2^32)
    const int k = (bid - b * gridDim.x) * OD_WAVES + wave;  // slot: level l owns [kpBase_l, kpBase_l + nDesired_l)
    // wave-uniform record: x, y and the window base live in SGPRs (its load first: the window's
    // address depends on it)
    const int kc = min(k, g.kpCap - 1);
    // (32-bit element offsets into the per-slot arrays: the host checks B * kpCap * 32 < 2^32)
    const uint32_t fslot = (uint32_t)b * (uint32_t)g.kpCap;
    const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)lvlOut[fslot + (uint32_t)kc]);
    // the slot's level: one byte of the host-built slot -> level table (a scalar load beside the
    // record's), then the frame's (first output slot, count) of that level (select_frame_done)
    const uint32_t lw = *(const uint32_t*)(slotLvl + (kc & ~3));
    const int l = (int)((lw >> (8 * (kc & 3))) & 0xFFu);
    const int2 linfo = lvlInfo[(uint32_t)b * ORB_MAX_LEVELS + (uint32_t)l];
    const LevelGeom& lg = g.lv[l];
    const int idx = k - lg.kpBase;
    // raw window: padded rows y-5 .. y+37 (level rows y-21 .. y+21), padded columns xa .. xa+63
    // (keypoints lie in 16 <= x <= w-7 and y likewise, App. B / DESIGN §4; the clamp only keeps
    // an empty slot's stale record inside the level; the last row's over-read stays inside the
    // pyramid's tail slack).  Loaded before the slot is known to be filled: the per-level counts
    // are scalar loads of their own
    const int x = min(max((int)(e & 0xFFF), 16), lg.w - 7), y = min(max((int)((e >> 12) & 0xFFF), 16), lg.h - 7);
    const int score = e >> 24;
    const int xa = (x - 5) & ~15;
    const uint4* src = (const uint4*)(pyr + lg.base + (long long)b * lg.fstride +
                                      (long long)(y + EDGE - OD_WR) * lg.pitch + xa);
    const uint32_t pu = (uint32_t)lg.pitch >> 4;
    uint8_t* W = s_buf[wave];
    uint32_t* Hs = (uint32_t*)s_buf[wave];
    uint32_t ico[5], ic10[5], ic01[5];  // IC_Angle: the lane's patch dwords and their coefficients
    i32x4v Bf[4];  // the row pass's B fragments (constant; in flight with the window loads)
    // (PC-relative addresses per table load: routing the tables through one opaque SGPR base
    // saved ~30 SALU per wave but let the loads sink below the window's, 0.420 -> 0.440 ms c3)
#pragma unroll
    for (int t = 0; t < 4; ++t) Bf[t] = __builtin_bit_cast(i32x4v, c_rowB[t * 64 + lane]);
#if OD_SB
    od_f16x8 Ac[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) Ac[v] = __builtin_bit_cast(od_f16x8, c_colA[v * 64 + lane]);
#endif
    constexpr int NU = (2 * OD_WR + 1) * 4;  // 172 16-byte units
    uint4 v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int i = lane + 64 * j, r = i >> 2, c = i & 3;
        v[j] = src[i < NU ? __umul24((uint32_t)r, pu) + c : 0u];
    }
    // the IC tables of this alignment (dword loads), in flight with the window
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int sh320 = 320 * ((x + 1 - xa) & 3);
        ico[j] = c_icoff[lane + 64 * j];
        ic10[j] = c_ic10[sh320 + lane + 64 * j];
        ic01[j] = c_ic01[sh320 + lane + 64 * j];
    }
    {
        // the window as i8 p - 128 (p ^ 0x80): the row pass's MFMA operand as it is, and IC_Angle's
        // sums unchanged (the disc is symmetric in u and v: sum u = sum v = 0 over it).  All 192
        // units stored (units >= 172 repeat unit 0 into the buffer's unused tail, before the
        // row-pass sums are written): no masked store
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int i = lane + 64 * j;
            const uint4 w = make_uint4(v[j].x ^ 0x80808080u, v[j].y ^ 0x80808080u, v[j].z ^ 0x80808080u,
                                       v[j].w ^ 0x80808080u);
            ((uint4*)W)[(i >> 2) * (OD_WP / 16) + (i & 3)] = w;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS is in order per wave; compiler fence
    // IC_Angle (ORBextractor.cc:124-151): the disc sums m10 = sum u*I, m01 = sum v*I over
    // |u| <= umax[|v|], one patch dword per lane and step (patch row v = window row v + 21,
    // patch dword c = window dword pd0 + c): two v_dot4_i32_i8 of the window dword (p - 128)
    // with the dword's coefficient bytes (0 outside the disc).  sum u (p - 128) = sum u p since
    // sum u = 0 over the symmetric disc (likewise v): exact integer sums, any order.
    int m01 = 0, m10 = 0;
    {
        const int pc = x + 1 - xa;  // window column of patch column u = -15
        const uint8_t* P0 = W + (OD_WR - HALF_PATCH) * OD_WP + 4 * (pc >> 2);  // the patch's first dword
        // five full 64-lane steps: dwords n >= 279 (patch rows 31 .. 35, still inside the
        // 43-row window) carry zero coefficients, so no lane is masked off
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int pm = *(const int*)(P0 + ico[j]);
            m10 = __builtin_amdgcn_sdot4(pm, (int)ic10[j], m10, false);
            m01 = __builtin_amdgcn_sdot4(pm, (int)ic01[j], m01, false);
        }
    }
    // output position: level-major order (ORBextractor.cc:749-778)
    const int before = linfo.x, cntL = linfo.y;
    // an empty slot's wave does no work but stays for the workgroup's two barriers
    const bool active = k < g.kpCap && idx < cntL;  // wave-uniform
#if OD_SB
    const bool sbT = x + 18 < lg.xsimd_blur;  // no sample reaches the scalar tail: the shared blur
    const int sbO0 = x - 5 - xa;
#endif
    // IC_Angle's sums, then the angle arithmetic (fastAtan2, glibc sincosf: ~100 VALU, a fifth of a
    // keypoint's) once per workgroup: wave 0's lanes 0 .. 3 for the four slots, between the
    // two barriers, while the other waves run their row passes
    m01 = wave_total(m01);
    m10 = wave_total(m10);
    typedef float f32x2v __attribute__((ext_vector_type(2)));
    // The rBRIEF pattern: points 8 lane .. 8 lane + 7 (tests 4 lane .. 4 lane + 3), pair q =
    // (x, y) of point 8 lane + q.  The rule of DESIGN §6.1, as code: eight fully coalesced
    // dwordx2 rows of the pair-major table (each instruction reads 512 contiguous bytes, four
    // cache lines no other pattern load touches; the float4 form read all 32 lines of the table
    // with each of its four instructions, 64-B lane stride, and returned wrong data), issued by
    // one asm statement and waited by another before the first sample (the registers are outputs
    // of the first and in-out operands of the second: the compiler can neither move the loads nor
    // read the registers early).  OD_PAT_EARLY 1: issued by the active waves once their own row
    // pass is done, in flight across the second barrier; 2: before the first barrier (in flight
    // across both, 16 more VGPRs live through the row pass); 0: after the second barrier.
#ifndef OD_PAT_EARLY
#define OD_PAT_EARLY 1
#endif
#ifndef OD_PAT_SPLIT
#define OD_PAT_SPLIT 1  // 0: the wait inside the issuing asm (441 vs 427 us c3 for the float4 form)
#endif
    f32x2v pat[8];
    auto issue_pattern = [&]() {
        const uint32_t poff = 8u * (uint32_t)lane;
        asm volatile(
            "global_load_dwordx2 %0, %8, %9\n\t"
            "global_load_dwordx2 %1, %8, %9 offset:512\n\t"
            "global_load_dwordx2 %2, %8, %9 offset:1024\n\t"
            "global_load_dwordx2 %3, %8, %9 offset:1536\n\t"
            "global_load_dwordx2 %4, %8, %9 offset:2048\n\t"
            "global_load_dwordx2 %5, %8, %9 offset:2560\n\t"
            "global_load_dwordx2 %6, %8, %9 offset:3072\n\t"
            "global_load_dwordx2 %7, %8, %9 offset:3584"
#if !OD_PAT_SPLIT
            "\n\ts_waitcnt vmcnt(0)"
#endif
            : "=&v"(pat[0]), "=&v"(pat[1]), "=&v"(pat[2]), "=&v"(pat[3]), "=&v"(pat[4]), "=&v"(pat[5]),
              "=&v"(pat[6]), "=&v"(pat[7])
            : "v"(poff), "s"((const float*)c_patternf)
            : "memory");
    };
    if (lane == 0) s_mom[wave] = make_int2(m01, m10);
#if OD_PAT_EARLY == 2
    if (active) issue_pattern();
#endif
    lds_barrier();
    if (wave == 0 && lane < OD_WAVES) {
        const int2 mm = s_mom[lane];
        const float ang = fast_atan2((float)mm.x, (float)mm.y);
        // computeOrbDescriptor (ORBextractor.cc:155-194)
        const float factorPI = (float)(3.14159265358979323846 / 180.f);
        float sa, ca;
        glibc_sincosf(ang * factorPI, &sa, &ca);
        s_trig[lane] = make_float4(ang, sa, ca, 0.f);
    }
    // row pass on the matrix cores: for M-tile m (window rows kOdRow[m] .. +15) and N-tile t
    // (output columns n = 16t .. 16t+15 of the window), H = A x B with A = the window bytes as
    // i8 (p ^ 0x80 = p - 128) and B = the banded tap matrix B[k][n] = tap[k - n] (c_rowB), one
    // v_mfma_i32_16x16x64_i8 over all 64 window columns.  Columns 61 .. 63 (never inside a
    // needed band: sum column hc reads window columns o0 + hc .. o0 + hc + 6 <= 60) carry
    // (127, 127, 11) in A and (127, 127, 58) in B: + 32896 = 128 * 257 restores the unsigned
    // sum, so H = sum tap * p exactly (0 .. 65535).  Lane l holds H of column 16t + (l & 15),
    // rows kOdRow[m] + 4(l >> 4) .. +3: two row-pair dwords Hs[pair][n] (56 columns per pair
    // row, so 8 work-groups fit a CU; the column pass adds o0).  All window reads are issued before the first write (LDS
    // is in order per wave), so the sums overlay the window.
    if (active) {
        const int r16 = lane & 15, h4 = lane >> 4;
        const uint4* W4 = (const uint4*)W;
        uint4 A[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) A[m] = W4[(kOdRow[m] + r16) * (OD_WP / 16) + h4];
        const uint32_t keep = h4 == 3 ? 0x000000FFu : 0xFFFFFFFFu;
        const uint32_t bias = h4 == 3 ? 0x0B7F7F00u : 0u;
        const i32x4v zero = {0, 0, 0, 0};
#if OD_SB
        // Shared blur: the row pass per N-tile t as below, then the column pass on the matrix cores
        // too: D[o][n] = sum_k A[o][k] S[k][n] with S = the tile's row-pass sums split into bytes
        // (each byte an f16 denormal b * 2^-24: its bits, no conversion) and A = the banded taps
        // (x 256 for the high bytes, c_colA): D = T * 2^-24 exactly (f32, T < 2^24).  Out rows
        // o = 0 .. 43 in blocks 0 / 16 / 28 (= the row pass's M-tiles; rows 28 .. 31 twice, rows
        // 37 .. 43 partial and never read).  cvRound half-to-even of T / 65536 by the magic add,
        // saturated, four rows per dword into the column-major blurred window (OD_SBP dwords per
        // column).  Wave-uniform: keypoints whose samples reach the scalar tail take the sparse
        // path below.
        if (sbT) {
            i32x4v a[3];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                a[m].x = (int)A[m].x;
                a[m].y = (int)A[m].y;
                a[m].z = (int)A[m].z;
                a[m].w = (int)((A[m].w & keep) | bias);
            }
            const od_f32x4 zf = {0.f, 0.f, 0.f, 0.f};
            uint32_t* cb = (uint32_t*)W + r16 * OD_SBP + h4;
            auto pack = [&](const i32x4v& c) {  // rows 4h .. 4h+3: low bytes, then high bytes
                uint4 u;
                u.x = __builtin_amdgcn_perm((uint32_t)c.y, (uint32_t)c.x, 0x0c040c00u);
                u.y = __builtin_amdgcn_perm((uint32_t)c.w, (uint32_t)c.z, 0x0c040c00u);
                u.z = __builtin_amdgcn_perm((uint32_t)c.y, (uint32_t)c.x, 0x0c050c01u);
                u.w = __builtin_amdgcn_perm((uint32_t)c.w, (uint32_t)c.z, 0x0c050c01u);
                return __builtin_bit_cast(od_f16x8, u);
            };
            auto emit = [&](const od_f32x4& D, uint32_t* dst) {
                // (scalar fmas: this compiler folds a <2 x float> fma with splat constants into
                // the low lane's result copied to both lanes, see the samples' magic add)
                const uint32_t r0 = __builtin_bit_cast(uint32_t, __builtin_fmaf(D.x, 256.0f, 12582912.0f));
                const uint32_t r1 = __builtin_bit_cast(uint32_t, __builtin_fmaf(D.y, 256.0f, 12582912.0f));
                const uint32_t r2 = __builtin_bit_cast(uint32_t, __builtin_fmaf(D.z, 256.0f, 12582912.0f));
                const uint32_t r3 = __builtin_bit_cast(uint32_t, __builtin_fmaf(D.w, 256.0f, 12582912.0f));
                const uint32_t p01 = __builtin_amdgcn_perm(r1, r0, 0x05040100u);
                const uint32_t p23 = __builtin_amdgcn_perm(r3, r2, 0x05040100u);
                const u16x2 cap = {255, 255};
                const uint32_t s01 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, p01), cap));
                const uint32_t s23 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, p23), cap));
                *dst = __builtin_amdgcn_perm(s23, s01, 0x06040200u);
            };
            const int nt = sbO0 <= 8 ? 3 : 4;  // N-tiles covering sum columns o0 .. o0 + 39
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t == 3 && nt == 3) break;
                const od_f16x8 S0 = pack(__builtin_amdgcn_mfma_i32_16x16x64_i8(a[0], Bf[t], zero, 0, 0, 0));
                const od_f16x8 S1 = pack(__builtin_amdgcn_mfma_i32_16x16x64_i8(a[1], Bf[t], zero, 0, 0, 0));
                od_f32x4 D0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ac[0], S0, zf, 0, 0, 0);
                D0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ac[1], S1, D0, 0, 0, 0);
                const od_f16x8 S2 = pack(__builtin_amdgcn_mfma_i32_16x16x64_i8(a[2], Bf[t], zero, 0, 0, 0));
                od_f32x4 D1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ac[0], S1, zf, 0, 0, 0);
                D1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ac[2], S2, D1, 0, 0, 0);
                const od_f32x4 D2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ac[0], S2, zf, 0, 0, 0);
                uint32_t* ct = cb + 16 * t * OD_SBP;
                emit(D0, ct);
                emit(D1, ct + 4);
                emit(D2, ct + 7);
            }
        } else
#endif
        {
        uint32_t* q3 = Hs + 2 * h4 * OD_HN + r16 + (r16 >= 8 ? 32 : 48);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            i32x4v a;
            a.x = (int)A[m].x;  // the window is stored as p ^ 0x80
            a.y = (int)A[m].y;
            a.z = (int)A[m].z;
            a.w = (int)((A[m].w & keep) | bias);
            i32x4v c[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t], zero, 0, 0, 0);
            uint32_t* q = Hs + (kOdRow[m] / 2 + 2 * h4) * OD_HN + r16;
            // N-tile 3 first: its columns 56 .. 63 (beyond the 56-column pair rows) go to the
            // lane's own tile-2 slots, which tile 2 then overwrites (same lane, program order)
            q3[0] = (uint32_t)c[3].x | ((uint32_t)c[3].y << 16);
            q3[OD_HN] = (uint32_t)c[3].z | ((uint32_t)c[3].w << 16);
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                q[16 * t] = (uint32_t)c[t].x | ((uint32_t)c[t].y << 16);
                q[16 * t + OD_HN] = (uint32_t)c[t].z | ((uint32_t)c[t].w << 16);
            }
            q3 += (kOdRow[m + (m < 2)] - kOdRow[m]) / 2 * OD_HN;
        }
        }
    }
#if OD_PAT_EARLY == 1
    if (active) issue_pattern();
#endif
    lds_barrier();  // s_trig is written (and the row-pass sums: LDS)
    if (!active) return;
#if !OD_PAT_EARLY
    issue_pattern();
#endif
    const float4 trig = s_trig[wave];
    const float angle = trig.x, a = trig.z, bsin = trig.y;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the row-pass sums are in LDS
    // wave-uniform: can any sample leave the ROI (raw border bytes) or reach the scalar tail?
    const bool edge = x - 18 < 0 || x + 18 >= lg.w || y - 18 < 0 || y + 18 >= lg.h;
    const bool tailAny = x + 18 >= lg.xsimd_blur;
    const int o0 = x - 5 - xa;  // window column of sum column hc = 0 (level column x - 18)
    // Sample offsets: dy = cvRound(fma(px, b, py * a)), dx = cvRound(fma(px, a, -(py * b)))
    // (ORBextractor.cc:168-169 as g++ contracts them) on packed f32 pairs; cvRound = round half
    // to even of the float, taken as the low bits of v + (1.5 * 2^23 + 18) (one more RNE
    // rounding, exact for |v| < 2^22; the even addend keeps the tie parity), so the bits are
    // kMagic + dy + 18 = kMagic + r0 (window row of the first tap) and kMagic + dx + 18.
    constexpr uint32_t kMagic = 0x4B400000u;
    const f32x2v rA = {a, -bsin}, rB = {bsin, a};
    // tap words of the column pass for even / odd r0, opaque so they stay in VGPRs
    uint32_t tE0 = GP_E0, tE1 = GP_E1, tE2 = GP_E2, tE3 = GP_E3;
    uint32_t tO0 = GP_O0, tO1 = GP_O1, tO2 = GP_O2, tO3 = GP_O3;
    asm volatile("" : "+v"(tE0), "+v"(tE1), "+v"(tE2), "+v"(tE3), "+v"(tO0), "+v"(tO1), "+v"(tO2), "+v"(tO3));
    // sum (pair p, column dx + 18 + o0) = hbase[56 p + bits_x] (32-bit LDS addresses wrap); the
    // pair index p = r0 >> 1 comes from v_mul_u32_u24 of by >> 1, whose low 24 bits are
    // ((kMagic >> 1) & 0xFFFFFF) + p: that constant is taken off the base
    const uint32_t* hbase = Hs + (o0 - (int)kMagic) - (int)(OD_HN * ((kMagic >> 1) & 0xFFFFFFu));
    const uint32_t hb = (uint32_t)((const uint8_t*)hbase - s_buf[0]);  // as a byte offset from s_buf
    // tail columns (scalar-tail rounding): x + dx >= xsimd_blur <=> bits_x >= thr
    const uint32_t thr = kMagic + 18u + (uint32_t)(lg.xsimd_blur - x);
    uint32_t bxs[8], bys[8];
    int vals[8];
#if OD_PAT_SPLIT
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(pat[0]), "+v"(pat[1]), "+v"(pat[2]), "+v"(pat[3]), "+v"(pat[4]), "+v"(pat[5]), "+v"(pat[6]),
                   "+v"(pat[7])::"memory");
#endif
    // one copy of the loop per wave-uniform tail case (no per-sample tail test when none)
    auto samples = [&](auto tailC) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        // R = (fma(px, b, py * a), fma(px, a, py * -b)) with px / py splat from the loaded pair
        // by op_sel (no copies): v_pk_mul_f32 takes py (the high half) for both lanes, v_pk_fma_f32
        // px (the low half) for both
        f32x2v R;
        asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_fma_f32 %0, %1, %3, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]"
            : "=&v"(R)
            : "v"(pat[q]), "v"(rA), "v"(rB));
        // (the magic add per element: this compiler turns a <2 x float> add of a splat literal
        // into the low lane's sum copied to both lanes)
        const uint32_t by = __builtin_bit_cast(uint32_t, R.x + 12582930.0f);
        const uint32_t bx = __builtin_bit_cast(uint32_t, R.y + 12582930.0f);
        bxs[q] = bx;
        bys[q] = by;
        // byte offset (by >> 1) * 224 + 4 bx: v_lshl_add_u32 + v_mad_u32_u24 (the compiler's
        // mul / shift / add3 was one more)
        uint32_t hoff;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(hoff) : "v"(by >> 1), "v"(4u * OD_HN), "v"((bx << 2) + hb));
        const uint32_t* hq = (const uint32_t*)(s_buf[0] + hoff);
        // odd r0: the first pair starts one row early (taps shifted by one u16 lane)
        const uint32_t om = (uint32_t)__builtin_amdgcn_sbfe((int)by, 0, 1);
        const uint32_t t0 = bfi(om, tO0, tE0), t1 = bfi(om, tO1, tE1);
        const uint32_t t2 = bfi(om, tO2, tE2), t3 = bfi(om, tO3, tE3);
        const uint32_t T = dot2u(hq[3 * OD_HN], t3, dot2u(hq[2 * OD_HN], t2, dot2u(hq[OD_HN], t1, dot2u(hq[0], t0, 0u))));
        vals[q] = (int)blur_round(T, decltype(tailC)::value && bx >= thr);
    }
    };
#if OD_SB
    if (sbT) {
        // the blurred window's byte (column o0 + bits_x - kMagic, row bits_y - kMagic): one
        // v_mad_u32_u24 of the low 24 bits of bits_x, the constants folded into the base
        const uint32_t sbb = (uint32_t)(W - s_buf[0]) + (uint32_t)(4 * OD_SBP * o0) -
                             (uint32_t)(4 * OD_SBP) * (kMagic & 0xFFFFFFu) - kMagic;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            f32x2v R;
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_fma_f32 %0, %1, %3, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]"
                : "=&v"(R)
                : "v"(pat[q]), "v"(rA), "v"(rB));
            const uint32_t by = __builtin_bit_cast(uint32_t, R.x + 12582930.0f);
            const uint32_t bx = __builtin_bit_cast(uint32_t, R.y + 12582930.0f);
            bxs[q] = bx;
            bys[q] = by;
            uint32_t boff;
            asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(boff) : "v"(bx), "v"(4u * OD_SBP), "v"(by + sbb));
            vals[q] = s_buf[0][boff];
        }
    } else
#endif
    if (tailAny)
        samples(std::true_type{});
    else
        samples(std::false_type{});
    if (edge) {  // samples outside the ROI read the padded level itself (the window is overlaid)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int X = x + (int)(bxs[q] - kMagic) - 18, Y = y + (int)(bys[q] - kMagic) - 18;
            if (X < 0 || X >= lg.w || Y < 0 || Y >= lg.h)
                vals[q] = pyr[lg.base + (long long)b * lg.fstride + (long long)(Y + EDGE) * lg.pitch + (X + EDGE)];
        }
    }
    int nib = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) nib |= (vals[2 * q] < vals[2 * q + 1]) << q;
    const int other = lane_xor1(nib);
    const uint32_t kslot = fslot + (uint32_t)(before + idx);
    if ((lane & 1) == 0) desc[kslot * 32u + (uint32_t)(lane >> 1)] = (uint8_t)(nib | (other << 4));
    if (lane == 0) {
        orb_keypoint_t kp;
        kp.x = l == 0 ? (float)x : (float)x * lg.scale;
        kp.y = l == 0 ? (float)y : (float)y * lg.scale;
        kp.size = lg.size;
        kp.angle = angle;
        kp.response = lvlResp ? lvlResp[fslot + (uint32_t)k] : (float)score;
        kp.octave = l;
        kp.class_id = -1;
        kps[kslot] = kp;
    }
}
#endif  // ORB_TU_MAIN

// The descriptor image of one level (blurred ROI + raw border), over level coordinates
// [-3, ringX1) x [-3, ringY1), by the same row / column passes and rounding as k_orient_desc:
// test hook behind orb_debug_blur_image (not on the product path).  One thread per pixel.
#if ORB_TU_MAIN
__global__ void __launch_bounds__(256) k_debug_desc_image(const uint8_t* __restrict__ pyr, LevelGeom lg, int b,
                                                          uint8_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int W = lg.w + 2 * EDGE;
    const int X = i % W - EDGE, Y = i / W - EDGE;
    if (Y + EDGE >= lg.h + 2 * EDGE) return;
    const uint8_t* P = pyr + lg.base + (long long)b * lg.fstride;
    uint32_t v = P[(long long)(Y + EDGE) * lg.pitch + X + EDGE];
    if (X >= 0 && X < lg.w && Y >= 0 && Y < lg.h) {
        uint32_t T = 0;
        const int kk[7] = {18, 34, 49, 55, 49, 34, 18};
        for (int j = 0; j < 7; ++j) {
            uint32_t H = 0;
            for (int q = 0; q < 7; ++q) H += kk[q] * P[(long long)(Y + j - 3 + EDGE) * lg.pitch + X + q - 3 + EDGE];
            T += kk[j] * H;
        }
        v = blur_round(T, X >= lg.xsimd_blur);
    }
    out[i] = (uint8_t)v;
}
#endif  // ORB_TU_MAIN

// ---- SearchForInitialization ------------------------------------------------------------
struct MatchGeom {
    int minX, maxX, minY, maxY;
    float invW, invH;  // FRAME_GRID_COLS / (maxX - minX), FRAME_GRID_ROWS / (maxY - minY)
};

// One workgroup (KM_THREADS = 8 waves) per frame pair.
//   phase 0  F2's octave-0, in-grid keypoints — the only possible candidates of
//            GetFeaturesInArea(x, y, window, 0, 0) (Frame.cc:200-265) — are staged,
//            ranked by grid-traversal order (ix, iy, index: Frame.cc:233-258), so a slot
//            number IS the reference's candidate order; F1's octave-0 queries are listed in
//            index order.
//   phase 1  (parallel) every query's window candidates are scored; each keeps its 8
//            smallest keys (dist << KB | slot) = the reference's (distance, first-in-order).
//   phase 2  (one wave, sequential: vMatchedDistance / vnMatches21 feed later queries)
//            best = first candidate with vMatchedDistance > dist, second = the next such;
//            if a truncated top-8 holds < 2 such candidates the wave rescans the window.
//   phase 3  rotation histogram, ComputeThreeMaxima, vnMatches12 / vbPrevMatched out.
// Two instantiations of the same body, both run by k_match_init's workgroup of a pair:
//   <false>  every per-slot array in LDS (nmax octave-0 keypoints per frame, nmax <= 1024 by
//            the batch size, see orb_search_for_initialization_batch_device); a pair with more
//            returns true and is redone by
//   <true>   the large-capacity body (e.g. the reference init extractor at 1280x720:
//            nFeatures*2 = 5000, Tracking.cc:126/217, ~1086 level-0 keypoints): only the greedy
//            state (vMatchedDistance / vnMatches21, vnMatches12, bins) stays in LDS, the staged
//            descriptors / coordinates / top-8 lists live in the pair's global scratch slot
//            (L2-resident); up to 8192 keypoints per frame.
#define MATCH_TOPK 8
#ifndef KM_THREADS
#define KM_THREADS 512  // one workgroup (8 waves) per pair: at most a few pairs share a CU
#endif
#define KM_WIDE_PAIRS 256  // fewer pairs: 16-wave workgroups (phase 1: NT / 256 lanes per query)
#ifndef KM_WIDE_ALL
#define KM_WIDE_ALL 0  // 1: 16-wave workgroups (and the fixed-point phase 2) for every batch
#endif
#define MATCH_BIG_NMAX 8192
#ifndef KM_FIX
#define KM_FIX 1  // 0: the sequential (speculated) phase 2 for every launch
#endif
#ifndef KM_WIDE_PHASE0
#define KM_WIDE_PHASE0 1  // phase 0's compaction by the whole workgroup (every launch)
#endif
#ifndef KM_EARLY_BATCH
#define KM_EARLY_BATCH 1  // the staging reads ahead of the ranking in 8-wave launches too
#endif
#ifndef KM_FIX_BATCH
#define KM_FIX_BATCH 0  // 1: the fixed point in the batched (8-wave) launches too
#endif
#ifndef KM_TIMING  // 1: per-phase s_memrealtime sums of k_match_init's pairs (experiment builds only)
#define KM_TIMING 0
#endif
#if KM_TIMING
#if ORB_TU_MAIN
__device__ unsigned long long g_kmtime[8];
#endif
#define KM_T(i) const unsigned long long kmt##i = __builtin_amdgcn_s_memrealtime()
#else
#define KM_T(i)
#endif
// Insert key into the sorted list t, keeping the smallest entries: the new t[i] is the median
// of (old t[i-1], key, old t[i]) -- one v_med3_u32 per entry, all independent (the min / max
// insertion chain was two dependent ops per entry)
__device__ __forceinline__ void topk_insert(uint32_t (&t)[MATCH_TOPK], uint32_t key) {
#pragma unroll
    for (int i = MATCH_TOPK - 1; i >= 1; --i) {
        uint32_t r;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(t[i - 1]), "v"(key), "v"(t[i]));
        t[i] = r;
    }
    t[0] = min(t[0], key);
}

struct MatchArgs {
    const orb_keypoint_t* kps;
    const uint8_t* desc;
    const int* counts;
    int cap, nmax;
    const int* pf1;
    const int* pf2;
    MatchGeom mg;
    float nnratio;
    int checkOri;
    float r;
    float* prev;
    int* m12out;
    int* nmOut;
    int P;
    int* done;    // host call (P == 1): pinned flag the kernel sets to doneSeq once its outputs are
    int doneSeq;  // visible to the host (the caller spins on it instead of a stream synchronisation)
    int fixOff;   // LDS byte offset of the fixed-point phase 2's arrays (16-wave launches), 0: sequential
};

// ORBmatcher.cc:664-670: the rotation's histogram bin (HISTO_LENGTH 30, factor 1/30)
__device__ __forceinline__ int rot_bin30(float rot) {
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / 30));
    if (bin == 30) bin = 0;
    return bin;
}

// Byte size of one global scratch slot of the large-capacity body (nmax slots / queries).
__host__ __device__ inline size_t match_big_slot_bytes(int cap, int nmax) {
    // d2 32 + x2,y2,a2,cell 16 per F2 slot; q2i,qx,qy,lcnt 16 per query; top-8 lists
    // (also phase 0's key scratch: max(cap, 8 nmax) u32)
    const size_t keys = (size_t)(cap > MATCH_TOPK * nmax ? cap : MATCH_TOPK * nmax);
    return ((size_t)nmax * 64 + keys * 4 + 255) & ~(size_t)255;
}

// Returns true (block-uniform) when the pair exceeded nmax and was left at -2 (-1 for BIG).
template <bool BIG, int NT>
__device__ __forceinline__ bool match_pair(const MatchArgs& A, int p, int nmax, uint8_t* __restrict__ smem,
                                           uint8_t* __restrict__ gs) {
    constexpr int KB = BIG ? 13 : 11;  // slot bits of a (distance, slot) key
    constexpr uint32_t SLOT = (1u << KB) - 1u;
    __shared__ int s_n2c, s_n1c;
    __shared__ int s_hist[32];
    __shared__ int s_ind[3];
    __shared__ int s_col[65];  // first slot of grid column cx (slots are in (cx, cy, index) order)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int cap = A.cap;
    const MatchGeom mg = A.mg;
    const float r = A.r, nnratio = A.nnratio;
    float* __restrict__ prev = A.prev;
    const int f1 = A.pf1[p], f2 = A.pf2[p];
    const int n1 = A.counts[f1], n2 = A.counts[f2];
    const orb_keypoint_t* K1 = A.kps + (long long)f1 * cap;
    const orb_keypoint_t* K2 = A.kps + (long long)f2 * cap;
    const uint32_t* D1 = (const uint32_t*)(A.desc + (long long)f1 * cap * 32);
    const uint32_t* D2 = (const uint32_t*)(A.desc + (long long)f2 * cap * 32);
    // per F2 slot: x = vMatchedDistance (low 16 bits, 0xFFFF = INT_MAX) | (vnMatches21 + 1) << 16,
    // y = the F2 keypoint index — one LDS read gives the greedy pass all it needs of a slot
    uint32_t* s_d2;
    uint2* s_st;
    float *s_x2, *s_y2, *s_qx, *s_qy, *s_a2, *s_qa = nullptr;
    int *s_cell, *s_q2i, *s_lcnt, *s_m12;
    uint32_t* s_list;
    short* s_bslot;
    if constexpr (!BIG) {
        s_d2 = (uint32_t*)smem;  // nmax x 8
        s_st = (uint2*)(s_d2 + (size_t)nmax * 8);
        s_x2 = (float*)(s_st + nmax);
        s_y2 = s_x2 + nmax;
        s_cell = (int*)(s_y2 + nmax);  // posX * 48 + posY
        s_q2i = s_cell + nmax;         // query -> i1
        s_qx = (float*)(s_q2i + nmax);
        s_qy = s_qx + nmax;
        s_a2 = s_qy + nmax;                       // F2 slot angle
        s_qa = s_a2 + nmax;                       // query angle (the F1 keypoint's)
        s_list = (uint32_t*)(s_qa + nmax);        // nmax x TOPK
        s_lcnt = (int*)(s_list + (size_t)nmax * MATCH_TOPK);
        s_m12 = s_lcnt + nmax;                    // vnMatches12 (cap)
        s_bslot = (short*)(s_m12 + cap);          // F2 slot of each accepted i1 (cap)
    } else {
        s_st = (uint2*)smem;                      // LDS: greedy state
        s_m12 = (int*)(s_st + nmax);
        s_bslot = (short*)(s_m12 + cap);
        s_d2 = (uint32_t*)gs;                     // global scratch slot
        s_x2 = (float*)(s_d2 + (size_t)nmax * 8);
        s_y2 = s_x2 + nmax;
        s_cell = (int*)(s_y2 + nmax);
        s_a2 = (float*)(s_cell + nmax);
        s_q2i = (int*)(s_a2 + nmax);
        s_qx = (float*)(s_q2i + nmax);
        s_qy = s_qx + nmax;
        s_lcnt = (int*)(s_qy + nmax);
        s_list = (uint32_t*)(s_lcnt + nmax);
    }
    uint32_t* s_key = s_list;  // phase-0 scratch (cap entries)
    KM_T(0);
    // ---- phase 0: keys in parallel, then ordered compaction ----
    // s_key[i2] = traversal key of F2 keypoint i2 or ~0 (not octave 0 / outside the grid);
    // s_m12[i1] = 1 if F1 keypoint i1 is a query (octave 0), as scratch.
    for (int i = tid; i < n2; i += NT) {
        const orb_keypoint_t kp = K2[i];
        const int px = (int)roundf((kp.x - mg.minX) * mg.invW);
        const int py = (int)roundf((kp.y - mg.minY) * mg.invH);
        const bool ok = kp.octave == 0 && !(px < 0 || px >= 64 || py < 0 || py >= 48);
        s_key[i] = ok ? (((uint32_t)(px * 48 + py) << 16) | (uint32_t)i) : 0xFFFFFFFFu;
    }
    for (int i = tid; i < n1; i += NT) s_m12[i] = K1[i].octave == 0;  // level1 > 0 -> continue (ORBmatcher.cc:615)
    if constexpr (BIG) __threadfence_block();
    __syncthreads();
    if constexpr (!BIG && KM_WIDE_PHASE0) {
        // both lists compacted by the whole workgroup, NT entries per round (per wave a ballot
        // count, the waves' offsets from a table of NT / 64); the single-wave loops below took
        // ~2.6 us per pair alone
        __shared__ int s_wc2[16], s_wc1[16];
        int base2 = 0, base1 = 0;
        for (int i0 = 0; i0 < max(n1, n2); i0 += NT) {
            const int i = i0 + tid;
            const uint32_t key = i < n2 ? s_key[i] : 0xFFFFFFFFu;
            const bool ok2 = key != 0xFFFFFFFFu;
            const bool ok1 = i < n1 && s_m12[i];
            const uint64_t m2 = __ballot(ok2), m1 = __ballot(ok1);
            if (lane == 0) {
                s_wc2[wave] = __popcll(m2);
                s_wc1[wave] = __popcll(m1);
            }
            __syncthreads();  // (also: every read of s_key's round precedes the writes below)
            int o2 = base2, o1 = base1, t2 = 0, t1 = 0;
            for (int w = 0; w < NT / 64; ++w) {
                const int c2 = s_wc2[w], c1 = s_wc1[w];
                if (w < wave) o2 += c2, o1 += c1;
                t2 += c2;
                t1 += c1;
            }
            if (ok2) s_key[o2 + lanes_below(m2)] = key;
            if (ok1 && o1 + lanes_below(m1) < nmax) s_q2i[o1 + lanes_below(m1)] = i;
            base2 += t2;
            base1 += t1;
            __syncthreads();
        }
        if (tid == 0) {
            s_n2c = base2;
            s_n1c = base1;
        }
    } else if (wave == 0) {  // in-place, in-order compaction (one wave: reads precede writes)
        int base = 0;
        for (int i0 = 0; i0 < n2; i0 += 64) {
            const uint32_t key = i0 + lane < n2 ? s_key[i0 + lane] : 0xFFFFFFFFu;
            const bool ok = key != 0xFFFFFFFFu;
            const uint64_t m = __ballot(ok);
            if (ok) s_key[base + lanes_below(m)] = key;
            base += __popcll(m);
        }
        if (lane == 0) s_n2c = base;
    } else if (wave == 1) {
        int base = 0;
        for (int i0 = 0; i0 < n1; i0 += 64) {
            const int i1 = i0 + lane;
            const bool ok = i1 < n1 && s_m12[i1];
            const uint64_t m = __ballot(ok);
            if (ok && base + lanes_below(m) < nmax) s_q2i[base + lanes_below(m)] = i1;
            base += __popcll(m);
        }
        if (lane == 0) s_n1c = base;
    }
    if constexpr (BIG) __threadfence_block();
    __syncthreads();
    const int n2c = s_n2c, n1c = s_n1c;
    if (n2c > nmax || n1c > nmax) {  // capacity exceeded: fall back / report, never truncate silently
        if (tid == 0) A.nmOut[p] = BIG ? -1 : -2;
        return true;
    }
    KM_T(1);
    // rank F2 candidates by traversal key -> slot.  16-wave launches with few candidates: LPK
    // adjacent lanes per key, each counting every LPK-th key, summed on DPP (one thread per key
    // counted all n2c keys).  Every global read of this stage (the candidates' records and
    // descriptors, the queries' records and positions, phase 1's query descriptors: host memory
    // in a host call) is issued before the counting, so their latencies overlap it and each other
    // instead of following one another (phase 1's then starts with its descriptors in registers;
    // with the med3 top-8 and the row-only window test, phase 1 11.2 -> 8.2 us per pair alone)
    int lpk = 1;
    if constexpr (!BIG && NT == 1024) lpk = n2c <= 256 ? 4 : n2c <= 512 ? 2 : 1;
    constexpr bool early = !BIG && (NT == 1024 || KM_EARLY_BATCH);
    uint32_t d1pre[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    orb_keypoint_t qkp{};
    float2 qprev = make_float2(0.f, 0.f);
    const bool qEarly = early && n1c <= NT && tid < n1c;
    if constexpr (early) {
        const int qP = tid / (NT / 256);  // phase 1's first round: NT / 256 lanes per query
        if (qP < n1c) {
            const int i1 = s_q2i[qP];
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                const uint4 v4 = ((const uint4*)D1)[(long long)i1 * 2 + w];
                d1pre[4 * w] = v4.x, d1pre[4 * w + 1] = v4.y, d1pre[4 * w + 2] = v4.z, d1pre[4 * w + 3] = v4.w;
            }
        }
        if (qEarly) {
            const int i1 = s_q2i[tid];
            qkp = K1[i1];
            if (prev) qprev = *(const float2*)(prev + ((long long)p * cap + i1) * 2);
        }
    }
    for (int t0 = tid; t0 < n2c * lpk; t0 += NT) {
        const int t = t0 / lpk, sub = t0 - t * lpk;  // (lpk divides NT: a key's lanes share a wave)
        const uint32_t k = s_key[t];
        const int i2 = (int)(k & 0xFFFF);
        orb_keypoint_t kp{};
        if (sub == 0) kp = K2[i2];
        uint32_t dv[8];
#pragma unroll
        for (int w = 0; w < 8; ++w)
            if (w % lpk == sub) dv[w] = D2[(long long)i2 * 8 + w];
        int rank = 0;
        for (int u = sub; u < n2c; u += lpk) rank += s_key[u] < k;
        if constexpr (early) {
            if (lpk >= 2) rank += __builtin_amdgcn_mov_dpp(rank, 0xB1, 0xF, 0xF, false);  // quad_perm xor 1
            if (lpk >= 4) rank += __builtin_amdgcn_mov_dpp(rank, 0x4E, 0xF, 0xF, false);  // quad_perm xor 2
        }
#pragma unroll
        for (int w = 0; w < 8; ++w)
            if (w % lpk == sub) s_d2[rank * 8 + w] = dv[w];
        if (sub != 0) continue;
        s_x2[rank] = kp.x;
        s_y2[rank] = kp.y;
        s_a2[rank] = kp.angle;
        s_cell[rank] = (int)(k >> 16);
        s_st[rank] = make_uint2(0xFFFFu, (uint32_t)i2);
    }
    if (qEarly) {
        s_qx[tid] = prev ? qprev.x : qkp.x;
        s_qy[tid] = prev ? qprev.y : qkp.y;
        if constexpr (!BIG) s_qa[tid] = qkp.angle;
    }
    if (!qEarly || !early)
        for (int q = (early && n1c <= NT) ? n1c : tid; q < n1c; q += NT) {
            const int i1 = s_q2i[q];
            const orb_keypoint_t kp = K1[i1];
            s_qx[q] = prev ? prev[((long long)p * cap + i1) * 2] : kp.x;
            s_qy[q] = prev ? prev[((long long)p * cap + i1) * 2 + 1] : kp.y;
            if constexpr (!BIG) s_qa[q] = kp.angle;  // (only queries are ever accepted)
        }
    if constexpr (BIG) __threadfence_block();
    __syncthreads();
    for (int i = tid; i < n1; i += NT) {
        s_m12[i] = -1;
        s_bslot[i] = -1;
    }
    if (tid <= 64) {  // lower_bound(s_cell, tid * 48): a window's columns are one slot range
        int lo = 0, hi = n2c;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_cell[mid] < tid * 48)
                lo = mid + 1;
            else
                hi = mid;
        }
        s_col[tid] = lo;
    }
    __syncthreads();
    // A slot in the window's column range [s_col[minCX], s_col[maxCX + 1]) already has its grid
    // column inside the window: only its grid row is tested, so the LDS body keeps the row alone
    // (no division by 48 per candidate)
    if constexpr (!BIG) {
        for (int j = tid; j < n2c; j += NT) s_cell[j] = s_cell[j] % 48;
        __syncthreads();
    }
    KM_T(2);
    // ---- phase 1: per-query top-8 (dist, order), two lanes per query (candidates j of one
    // parity each), their sorted lists merged on DPP ----
    for (int q0 = 0; q0 < n1c; q0 += NT / (NT / 256)) {
        const int q = q0 + tid / (NT / 256), sub = tid & ((NT / 256) - 1);
        const bool act = q < n1c;
        float qx = 0.f, qy = 0.f;
        int minCX = 1, maxCX = 0, minCY = 1, maxCY = 0;
        uint32_t d1[8] = {};
        if (act) {
            qx = s_qx[q];
            qy = s_qy[q];
            minCX = max(0, (int)floorf((qx - mg.minX - r) * mg.invW));
            maxCX = min(63, (int)ceilf((qx - mg.minX + r) * mg.invW));
            minCY = max(0, (int)floorf((qy - mg.minY - r) * mg.invH));
            maxCY = min(47, (int)ceilf((qy - mg.minY + r) * mg.invH));
            if (early && q0 == 0) {
#pragma unroll
                for (int w = 0; w < 8; ++w) d1[w] = d1pre[w];
            } else {
                const int i1 = s_q2i[q];
#pragma unroll
                for (int w = 0; w < 2; ++w) {  // two 16-B loads (descriptor rows are 32-B aligned)
                    const uint4 v4 = ((const uint4*)D1)[(long long)i1 * 2 + w];
                    d1[4 * w] = v4.x, d1[4 * w + 1] = v4.y, d1[4 * w + 2] = v4.z, d1[4 * w + 3] = v4.w;
                }
            }
        }
        uint32_t top[MATCH_TOPK];
#pragma unroll
        for (int k = 0; k < MATCH_TOPK; ++k) top[k] = 0xFFFFFFFFu;
        int cnt = 0;
        // the window's grid columns only (an empty column range gives j0 >= j1)
        const int j0 = s_col[min(minCX, 64)], j1 = s_col[max(maxCX + 1, 0)];
        for (int j = j0 + sub; j < j1; j += (NT / 256)) {
            // every read of the candidate issued at once (one LDS round trip per candidate, not
            // three dependent ones behind the window tests; prefetching the next candidate's
            // reads one iteration ahead measured slower: 15.8 vs 13.6 us per pair alone)
            const int cell = s_cell[j];
            const float x2 = s_x2[j], y2 = s_y2[j];
            const uint4 da = *(const uint4*)(s_d2 + j * 8), db = *(const uint4*)(s_d2 + j * 8 + 4);
            if constexpr (BIG) {
                const int cx = cell / 48, cy = cell - cx * 48;
                if (cx < minCX || cx > maxCX || cy < minCY || cy > maxCY) continue;
            } else {
                if (cell < minCY || cell > maxCY) continue;  // (the grid row)
            }
            if (fabsf(x2 - qx) > r || fabsf(y2 - qy) > r) continue;
            const int dist = __popc(d1[0] ^ da.x) + __popc(d1[1] ^ da.y) + __popc(d1[2] ^ da.z) + __popc(d1[3] ^ da.w) +
                             __popc(d1[4] ^ db.x) + __popc(d1[5] ^ db.y) + __popc(d1[6] ^ db.z) + __popc(d1[7] ^ db.w);
            topk_insert(top, ((uint32_t)dist << KB) | (uint32_t)j);
            ++cnt;
        }
        // merge with the partner lanes' lists (DPP quad_perm xor 1, then xor 2): the 8 smallest
        // of two sorted lists are min(a[i], b[7-i]) (a bitonic sequence), sorted by a 3-stage
        // bitonic merge
        uint32_t m8[MATCH_TOPK];
#pragma unroll
        for (int k = 0; k < MATCH_TOPK; ++k) m8[k] = top[k];
        auto merge_round = [&](auto ctlC) {
            constexpr int ctl = decltype(ctlC)::value;
            cnt += __builtin_amdgcn_mov_dpp(cnt, ctl, 0xF, 0xF, false);
            uint32_t o[MATCH_TOPK];
#pragma unroll
            for (int k = 0; k < MATCH_TOPK; ++k) o[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)m8[MATCH_TOPK - 1 - k], ctl, 0xF, 0xF, false);
#pragma unroll
            for (int k = 0; k < MATCH_TOPK; ++k) m8[k] = min(m8[k], o[k]);
#pragma unroll
            for (int d = 4; d >= 1; d >>= 1)
#pragma unroll
                for (int k = 0; k < MATCH_TOPK; ++k)
                    if ((k & d) == 0) {
                        const uint32_t lo = min(m8[k], m8[k + d]), hi = max(m8[k], m8[k + d]);
                        m8[k] = lo;
                        m8[k + d] = hi;
                    }
        };
        merge_round(std::integral_constant<int, 0xB1>{});
        if constexpr ((NT / 256) == 4) merge_round(std::integral_constant<int, 0x4E>{});
        if (act && sub == 0) {
#pragma unroll
            for (int k = 0; k < MATCH_TOPK; ++k) s_list[q * MATCH_TOPK + k] = m8[k];
            s_lcnt[q] = cnt;
        }
    }
    if constexpr (BIG) __threadfence_block();
    __syncthreads();
    KM_T(3);
    // ---- phase 2: the sequential greedy pass (ORBmatcher.cc:611-680) on one wave ----
    // Speculated eight queries at a time (lane 8g + c: query q0 + g, candidate c of its top-8),
    // exact: query q's outcome is fixed by its best and second live candidates (the first two of
    // its sorted top-8 whose vMatchedDistance exceeds their distance), and an accepted query
    // changes exactly one slot (its best), lowering its vMatchedDistance.  So every query of the
    // batch is decided from the batch-start state unless an earlier query of the batch accepted
    // its best or second slot (a live slot can only die; a taken best is a steal), or it needs
    // the window rescan (a truncated top-8 with < 2 live candidates); the batch commits
    // its queries before the first such one (their slots are distinct, their vnMatches21
    // predecessors precede the batch) and the next batch starts there.  A rescan query heading
    // a batch runs alone on the whole wave.
    // the exact rescan of query q0's whole window, on all 64 lanes of wave 0 (a query whose
    // truncated top-8 holds fewer than two live candidates)
    // the exact rescan of query q0's whole window on all 64 lanes of a wave: the smallest live
    // key and the second-smallest live distance (live(j, dist): candidate slot j not excluded)
    auto rescan_best = [&](const int q0, auto&& live, uint32_t& gbOut, int& contribOut) {
        const int i1 = s_q2i[q0];
        const float qx = s_qx[q0], qy = s_qy[q0];
        const int minCX = max(0, (int)floorf((qx - mg.minX - r) * mg.invW));
        const int maxCX = min(63, (int)ceilf((qx - mg.minX + r) * mg.invW));
        const int minCY = max(0, (int)floorf((qy - mg.minY - r) * mg.invH));
        const int maxCY = min(47, (int)ceilf((qy - mg.minY + r) * mg.invH));
        uint32_t d1[8];
#pragma unroll
        for (int w = 0; w < 2; ++w) {  // two 16-B loads (descriptor rows are 32-B aligned)
            const uint4 v4 = ((const uint4*)D1)[(long long)i1 * 2 + w];
            d1[4 * w] = v4.x, d1[4 * w + 1] = v4.y, d1[4 * w + 2] = v4.z, d1[4 * w + 3] = v4.w;
        }
        uint32_t lb = 0xFFFFFFFFu;
        int ls = 0x7fffffff;
        const int j1 = s_col[max(maxCX + 1, 0)];
        for (int j = s_col[min(minCX, 64)] + lane; j < j1; j += 64) {
            const int cell = s_cell[j];
            if constexpr (BIG) {
                const int cx = cell / 48, cy = cell - cx * 48;
                if (cx < minCX || cx > maxCX || cy < minCY || cy > maxCY) continue;
            } else {
                if (cell < minCY || cell > maxCY) continue;  // (the grid row)
            }
            if (fabsf(s_x2[j] - qx) > r || fabsf(s_y2[j] - qy) > r) continue;
            const int dist = hamming256(d1, s_d2 + j * 8);
            if (!live(j, dist)) continue;
            const uint32_t key = ((uint32_t)dist << KB) | (uint32_t)j;
            if (key < lb) {
                if (lb != 0xFFFFFFFFu) ls = (int)(lb >> KB);
                lb = key;
            } else if (dist < ls) {
                ls = dist;
            }
        }
        uint32_t gb = lb;
        gb = wave_min_u32(gb);
        int contrib = (lb == gb) ? ls : (lb == 0xFFFFFFFFu ? 0x7fffffff : (int)(lb >> KB));
        contrib = (int)wave_min_u32((uint32_t)contrib);  // (non-negative)
        gbOut = gb;
        contribOut = contrib;
    };
    auto rescan_query = [&](const int q0) {
        uint32_t gb;
        int contrib;
        rescan_best(q0, [&](int j, int dist) { return (int)(s_st[j].x & 0xFFFFu) > dist; }, gb, contrib);
        if (gb == 0xFFFFFFFFu) return;
        const int i1 = s_q2i[q0];
        const int rDist = (int)(gb >> KB), rSlot = (int)(gb & SLOT);
        if (rDist <= 50 && (float)rDist < (float)contrib * nnratio && lane == 0) {
            const uint2 sb = s_st[rSlot];
            const int old = (int)(sb.x >> 16) - 1;
            if (old >= 0) s_m12[old] = -1;
            s_m12[i1] = (int)(sb.y & 0x1FFFu);
            s_st[rSlot].x = (uint32_t)rDist | ((uint32_t)(i1 + 1) << 16);
            s_bslot[i1] = (short)rSlot;
        }
    };
    // Phase 2 as a fixed point (the single-pair call, 16 waves, when its arrays fit the LDS):
    // query q's decision depends only on the earlier queries' acceptances -- candidate slot s is
    // live for q iff dist < MD_q(s) = min{d_j : j < q accepted s} (vMatchedDistance as q sees
    // it) -- so every query is decided in parallel from the previous iteration's acceptances
    // until they repeat; the sequential result is the unique fixed point and is reached (after
    // iteration k the first k queries are final; SearchByProjection(local)'s resolver, orb_match).
    // Up to three acceptors per slot and iteration (more: the sequential pass below decides).
    // Final: every accepting query keeps its slot (bins count the stolen ones too), the slot's
    // last acceptor owns the match (vnMatches21).
    bool fixDone = false;
    if constexpr (!BIG) {
        if (A.fixOff) {  // (the host enables it only when every query has a thread: nmax <= NT)
            __shared__ int s_fn, s_fch, s_fovf;
            uint32_t* faB[2];
            int* fcB[2];
            faB[0] = (uint32_t*)(smem + A.fixOff);
            faB[1] = faB[0] + 3 * nmax;
            fcB[0] = (int*)(faB[1] + 3 * nmax);
            fcB[1] = fcB[0] + nmax;
            int* fdec = fcB[1] + nmax;  // per query: (dist << 16) | slot, -1 none
            int* fnew = fdec + nmax;
            uint16_t* fres = (uint16_t*)(fnew + nmax);
            for (int i = tid; i < n2c; i += NT) fcB[0][i] = 0;
            for (int i = tid; i < n1c; i += NT) fdec[i] = -1;
            if (tid == 0) s_fovf = 0;
            const int q = tid;
            const bool qin = q < n1c;
            const int cnt = qin ? s_lcnt[q] : 0;
            uint32_t el[MATCH_TOPK];
#pragma unroll
            for (int k = 0; k < MATCH_TOPK; ++k) el[k] = qin ? s_list[q * MATCH_TOPK + k] : 0xFFFFFFFFu;
            int cur = 0;
            bool conv = false;
            for (int it = 0; it < n1c + 2 && !conv; ++it) {
                const uint32_t* fa = faB[cur];
                const int* fc = fcB[cur];
                uint32_t* na = faB[cur ^ 1];
                int* nc = fcB[cur ^ 1];
                for (int i = tid; i < n2c; i += NT) nc[i] = 0;
                if (tid == 0) {
                    s_fn = 0;
                    s_fch = 0;
                }
                __syncthreads();
                auto md = [&](int sl, int qq) {  // MD_qq(sl): 0xFFFF = INT_MAX
                    int m = 0xFFFF;
                    const int c = min(fc[sl], 3);
                    for (int i = 0; i < c; ++i) {
                        const uint32_t v = fa[3 * sl + i];
                        if ((int)(v >> 9) < qq) m = min(m, (int)(v & 511u));
                    }
                    return m;
                };
                int dec = -1;
                if (qin && cnt > 0) {
                    const int k = min(cnt, MATCH_TOPK);
                    uint32_t b1 = 0xFFFFFFFFu, b2 = 0xFFFFFFFFu;
#pragma unroll
                    for (int j = 0; j < MATCH_TOPK; ++j) {
                        if (j < k && b2 == 0xFFFFFFFFu) {
                            const uint32_t e = el[j];
                            if (md((int)(e & SLOT), q) > (int)(e >> KB)) {
                                if (b1 == 0xFFFFFFFFu)
                                    b1 = e;
                                else
                                    b2 = e;
                            }
                        }
                    }
                    if (cnt > MATCH_TOPK && b2 == 0xFFFFFFFFu) {
                        fres[atomicAdd(&s_fn, 1)] = (uint16_t)q;
                        dec = -2;
                    } else if (b1 != 0xFFFFFFFFu) {
                        const int bd = (int)(b1 >> KB);
                        const int second = b2 != 0xFFFFFFFFu ? (int)(b2 >> KB) : 0x7fffffff;
                        if (bd <= 50 && (float)bd < (float)second * nnratio) dec = (bd << 16) | (int)(b1 & SLOT);
                    }
                    if (dec >= 0) {
                        const int sl = dec & 0xFFFF;
                        const int ix = atomicAdd(&nc[sl], 1);
                        if (ix < 3)
                            na[3 * sl + ix] = ((uint32_t)q << 9) | (uint32_t)(dec >> 16);
                        else
                            s_fovf = 1;
                    }
                }
                if (qin && dec != -2) fnew[q] = dec;
                __syncthreads();
                const int nres = s_fn;
                for (int rr = wave; rr < nres; rr += NT / 64) {  // exact rescans, a wave each
                    const int qq = fres[rr];
                    uint32_t gb;
                    int contrib;
                    rescan_best(qq, [&](int j, int dist) { return md(j, qq) > dist; }, gb, contrib);
                    int d2 = -1;
                    if (gb != 0xFFFFFFFFu) {
                        const int rd = (int)(gb >> KB);
                        if (rd <= 50 && (float)rd < (float)contrib * nnratio) d2 = (rd << 16) | (int)(gb & SLOT);
                    }
                    if (lane == 0) {
                        fnew[qq] = d2;
                        if (d2 >= 0) {
                            const int sl = d2 & 0xFFFF;
                            const int ix = atomicAdd(&nc[sl], 1);
                            if (ix < 3)
                                na[3 * sl + ix] = ((uint32_t)qq << 9) | (uint32_t)(d2 >> 16);
                            else
                                s_fovf = 1;
                        }
                    }
                }
                __syncthreads();
                if (qin && fnew[q] != fdec[q]) {
                    fdec[q] = fnew[q];
                    s_fch = 1;
                }
                __syncthreads();
                conv = s_fch == 0 || s_fovf != 0;
                cur ^= 1;
                __syncthreads();  // s_fch / s_fovf read by every thread before the next reset
            }
            if (conv && s_fovf == 0) {
                fixDone = true;
                // (the lists of the last iteration, faB[cur] / fcB[cur], hold the final acceptances)
                const uint32_t* fa = faB[cur];
                const int* fc = fcB[cur];
                if (qin && fdec[q] >= 0) s_bslot[s_q2i[q]] = (short)(fdec[q] & 0xFFFF);
                for (int sl = tid; sl < n2c; sl += NT) {
                    const int c = min(fc[sl], 3);
                    int owner = -1;
                    for (int i = 0; i < c; ++i) owner = max(owner, (int)(fa[3 * sl + i] >> 9));
                    if (owner >= 0) s_m12[s_q2i[owner]] = (int)(s_st[sl].y & 0x1FFFu);
                }
            }
            __syncthreads();
        }
    }
    if (!fixDone && wave == 0 && n1c > 0) {
        const int grp = lane >> 3, cand = lane & 7;
        int q0 = 0;
        while (q0 < n1c) {
            const int q = q0 + grp;
            const bool qin = q < n1c;
            // the group's count, list entry and query index read together (one LDS round trip)
            const int qc = min(q, n1c - 1);
            const int cntR = s_lcnt[qc];
            const uint32_t eR = s_list[qc * MATCH_TOPK + cand];
            const int i1q = s_q2i[qc];
            const int cnt = qin ? cntR : 0;
            const int k = min(cnt, MATCH_TOPK);
            const uint32_t e = cand < k ? eR : 0xFFFFFFFFu;
            const uint2 st = cand < k ? s_st[e & SLOT] : make_uint2(0u, 0u);
            const bool valid = cand < k && (int)(st.x & 0xFFFFu) > (int)(e >> KB);
            // the group's best (smallest live key: the lists are sorted) and second, by 8-lane
            // min reductions on DPP (quad_perm xor 1, xor 2, row_half_mirror); the best lane
            // keeps its own slot state for the commit
            const uint32_t key = valid ? e : 0xFFFFFFFFu;
            const uint32_t best = min8(key);
            const uint32_t sec = min8(valid && e != best ? e : 0xFFFFFFFFu);
            const bool rescan = cnt > MATCH_TOPK && sec == 0xFFFFFFFFu;  // < 2 live in a truncated list
            const int second = sec != 0xFFFFFFFFu ? (int)(sec >> KB) : 0x7fffffff;
            const int bestDist = (int)(best >> KB), bestSlot = (int)(best & SLOT);
            const bool accept = best != 0xFFFFFFFFu && !rescan && bestDist <= 50 &&
                                (float)bestDist < (float)second * nnratio;
            // first query the batch-start state cannot decide
            const uint64_t accM = __ballot(accept && cand == 0);  // bit 8g: group g accepts
            // lane 8g + c checks group c's accepted slot against query g's best and second
            // (query g's decision reads only those two slots: the rescan test included, both
            // live means >= 2 live), one ds_bpermute for the eight groups' slots
            const int bsC = __shfl(bestSlot, 8 * cand, 64);
            const bool hit = cand < grp && ((accM >> (8 * cand)) & 1ull) &&
                             ((best != 0xFFFFFFFFu && bestSlot == bsC) || (sec != 0xFFFFFFFFu && (int)(sec & SLOT) == bsC));
            const uint64_t stopM = __ballot(hit || (rescan && cand == 0));
            const int jstop = stopM ? (__ffsll((unsigned long long)stopM) - 1) >> 3 : 8;
            if (accept && valid && e == best && grp < jstop) {
                // by the best candidate's lane; distinct slots: these writes commute, and the
                // next batch's reads follow them
                const int i1 = i1q;
                const int old = (int)(st.x >> 16) - 1;  // vnMatches21[bestIdx2]
                if (old >= 0) s_m12[old] = -1;
                s_m12[i1] = (int)(st.y & 0x1FFFu);
                s_st[bestSlot].x = (uint32_t)bestDist | ((uint32_t)(i1 + 1) << 16);
                s_bslot[i1] = (short)bestSlot;
            }
            if (jstop > 0) {
                q0 += jstop;
                continue;
            }
            rescan_query(q0);
            q0 += 1;
        }
    }
    __syncthreads();
    KM_T(4);
    // ---- phase 3 ----
    if (A.checkOri) {
        if (tid < 32) s_hist[tid] = 0;
        __syncthreads();
        // rotation bin of every accepted i1, the stolen ones included (ORBmatcher.cc:664-676); only
        // queries are ever accepted, so the LDS body walks its queries (angles from LDS: s_qa /
        // s_a2, the slot kept for the output pass); the histogram is a count, so order is free
        const int nw = BIG ? n1 : n1c;
        for (int t = tid; t < nw; t += NT) {
            const int i = BIG ? t : s_q2i[t];
            const int sl = s_bslot[i];
            if (sl < 0) continue;
            atomicAdd(&s_hist[rot_bin30((BIG ? K1[i].angle : s_qa[t]) - s_a2[sl])], 1);
        }
        __syncthreads();
        if (wave == 0) {
            // ComputeThreeMaxima (ORBmatcher.cc:1748-1789) on one wave: its strict-> insertion scan
            // keeps the three largest non-zero counts, ties in bin order, so the bins are the
            // three largest keys (count << 8 | 255 - bin) by wave-max reductions (tid 0 scanning
            // the 30 bins took ~1 us per pair)
            const int v = lane < 30 ? s_hist[lane] : 0;
            const uint32_t key = v > 0 ? ((uint32_t)v << 8) | (uint32_t)(255 - lane) : 0u;
            const uint32_t k1 = ~wave_min_u32(~key);
            const uint32_t k2 = ~wave_min_u32(~(key == k1 ? 0u : key));
            const uint32_t k3 = ~wave_min_u32(~(key == k1 || key == k2 ? 0u : key));
            const int max1 = (int)(k1 >> 8), max2 = (int)(k2 >> 8), max3 = (int)(k3 >> 8);
            int ind1 = k1 ? 255 - (int)(k1 & 255u) : -1, ind2 = k2 ? 255 - (int)(k2 & 255u) : -1;
            int ind3 = k3 ? 255 - (int)(k3 & 255u) : -1;
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1;
                ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
            if (lane == 0) {
                s_ind[0] = ind1;
                s_ind[1] = ind2;
                s_ind[2] = ind3;
            }
        }
        __syncthreads();
        const int i1x = s_ind[0], i2x = s_ind[1], i3x = s_ind[2];
        for (int t = tid; t < nw; t += NT) {
            const int i = BIG ? t : s_q2i[t];
            const int sl = s_bslot[i];
            if (sl < 0) continue;
            const int bn = rot_bin30((BIG ? K1[i].angle : s_qa[t]) - s_a2[sl]);
            if (bn != i1x && bn != i2x && bn != i3x) s_m12[i] = -1;
        }
        __syncthreads();
    }
    int nm = 0;
    for (int i = tid; i < n1; i += NT) {
        const int m = s_m12[i];
        A.m12out[(long long)p * cap + i] = m;
        if (m >= 0) {
            nm++;
            if (prev) {  // vbPrevMatched[i1] = F2.mvKeysUn[i2].pt: the accepted slot's staged position
                const int sl = s_bslot[i];
                prev[((long long)p * cap + i) * 2] = s_x2[sl];
                prev[((long long)p * cap + i) * 2 + 1] = s_y2[sl];
            }
        }
    }
    nm = wave_total(nm);
    if (lane == 0) s_hist[wave] = nm;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) t += s_hist[w];
        A.nmOut[p] = t;
    }
#if KM_TIMING
    KM_T(5);
    if (tid == 0 && !BIG) {
        atomicAdd(&g_kmtime[0], kmt1 - kmt0);  // phase 0: keys + compaction
        atomicAdd(&g_kmtime[1], kmt2 - kmt1);  // ranking + staging
        atomicAdd(&g_kmtime[2], kmt3 - kmt2);  // phase 1
        atomicAdd(&g_kmtime[3], kmt4 - kmt3);  // phase 2
        atomicAdd(&g_kmtime[4], kmt5 - kmt4);  // phase 3 + output
        atomicAdd(&g_kmtime[5], 1ull);
        atomicAdd(&g_kmtime[6], (unsigned long long)n1c);
        atomicAdd(&g_kmtime[7], (unsigned long long)n2c);
    }
#endif
    return false;
}

// One workgroup per pair.  A pair whose F1 queries or F2 candidates exceed the LDS capacity
// A.nmax is redone in the same workgroup by the large-capacity body (nmaxBig, up to 8192
// keypoints), its staged arrays in the pair's own slot of the global scratch `big` (null when
// cap <= A.nmax: nothing can overflow).  The dynamic LDS covers both bodies' needs, so no
// second launch and nothing per call beyond this kernel.
// NT threads: KM_THREADS (8 waves) when pairs share CUs; 16 waves when each pair has a CU to
// itself (fewer pairs than KM_WIDE_PAIRS, e.g. one SearchForInitialization call): phase 1 then
// scores each query with four lanes instead of two.
#if ORB_TU_MAIN
template <int NT>
__global__ void __launch_bounds__(NT) k_match_init(MatchArgs A, uint8_t* __restrict__ big, int nmaxBig) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int p = blockIdx.x;
    if (match_pair<false, NT>(A, p, A.nmax, smem, nullptr) && big) {
        __syncthreads();  // the static LDS (counts, bins) is reused
        match_pair<true, NT>(A, p, nmaxBig, smem, big + (size_t)p * match_big_slot_bytes(A.cap, nmaxBig));
    }
    if (A.done) {  // (a host call's single workgroup) every wave's output stores complete, the
                   // workgroup's writes made visible to the host (system-scope release), then the flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(A.done, A.doneSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
#endif  // ORB_TU_MAIN

// ======================================================================================
// host side
// ======================================================================================
#if ORB_TU_MAIN
#if ORB_ILP_SPLIT
// orb_ilp.hip's launchers of its k_pyr_stream / k_fast (library-internal)
__attribute__((visibility("hidden"))) void orb_ilp_init();
__attribute__((visibility("hidden"))) void orb_ilp_pyr_stream(int B, size_t lds, hipStream_t st, const uint8_t* imgs, int stride, long long fpitch,
                        uint8_t* pyr, const uint32_t* scol, const uint4* srows, const StreamLevel* slv,
                        const uint32_t* srounds, const StreamGeom& sg, int* cellCount, int nCells);
__attribute__((visibility("hidden"))) void orb_ilp_fast(int nTiles, int B, hipStream_t st, const uint8_t* pyr,
                                                       const Geom& g, const FastTile* tiles, uint32_t* cand,
                                                       int* cellCount);
#endif
namespace {

inline int cvRoundH(double v) { return (int)lrint(v); }
inline short satS16(int v) { return (short)std::min(std::max(v, -32768), 32767); }

// OpenCV 2.4 getGaussianKernel(7, 2, CV_32F) -> convertTo(CV_32S, 256).
void gaussian_taps7(int* k7) {
    double scale2X = -0.5 / (2.0 * 2.0), sum = 0;
    float cf[7];
    for (int i = 0; i < 7; ++i) {
        double x = i - 3.0;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; ++i) cf[i] = (float)(cf[i] * sum);
    for (int i = 0; i < 7; ++i) k7[i] = cvRoundH(cf[i] * 256.0f);
}

}  // namespace

struct orb_extractor {
    int nfeatures = 0;
    double scaleFactor = 1.2;  // double member, as in the reference (ORBextractor.h:62)
    int nlevels = 0, scoreType = 1, fastTh = 20, device = 0, maxBatch = 1;
    std::vector<float> mvScaleFactor, mvInvScaleFactor;
    std::vector<int> nDesired;
    int umax[16] = {};
    int kpCap = 0;
    hipStream_t stream = nullptr;      // the handle's own stream (host-buffer entry points)
    hipStream_t lastStream = nullptr;  // stream of the last launch on this handle's workspace
    bool lastValid = false;            // lastStream names a stream that ran a launch
    hipEvent_t evOrder = nullptr;      // orders a launch after the previous one on another stream
    int pyrBatch = 0;                  // frames whose pyramid phase 1 left in the workspace
    // geometry of the current frame size
    int W = 0, H = 0;
    Geom g{};
    int fastCl = FT_CL;  // orb_debug_set_fast_corner_list
    std::vector<CellGeom> cells;
    std::vector<int> rtab;
    size_t listLds = 0;  // k_select<.., false> (re-runs in k_rerun): the survivor lists only
    size_t cellLds = 0, selectLds = 0;  // a FAST(7) re-run's LDS (largest cell); k_select's
    size_t resizeLds[ORB_MAX_LEVELS] = {}, resizeLdsS[ORB_MAX_LEVELS] = {};
    int resizeTail = 0;           // first level of k_pyr_resize_tail (nlevels: none)
    int tailBufA = 0, tailBufB = 0;
    size_t tailLds = 0;
    // k_pyr_stream plan (build_stream_plan); streamOk false: per-level launches only
    bool streamOk = false;
    StreamGeom sgeom{};
    size_t streamLds = 0;
    int streamK0 = 0;
    uint32_t* d_scol = nullptr;
    uint4* d_srows = nullptr;
    StreamLevel* d_slv = nullptr;
    uint32_t* d_srounds = nullptr;
    // device workspace
    uint8_t* d_pyr = nullptr;
    FastTile* d_tiles = nullptr;
    int nTiles = 0;
    uint32_t* d_cand = nullptr;
    int* d_cellCount = nullptr;
    uint32_t* d_cand2 = nullptr;  // k_select scratch when a level's survivors exceed its LDS
    uint32_t* d_lvl = nullptr;
    int* d_lvlCount = nullptr;
    int2* d_lvlInfo = nullptr;     // [frame][ORB_MAX_LEVELS] (first output slot, count): k_select's last WG
    int* d_selDone = nullptr;      // [frame] k_select workgroups done (self-resetting, zero between launches)
    uint8_t* d_slotLvl = nullptr;  // keypoint slot -> level (kpCap bytes, padded to a dword)
    uint64_t* d_candH = nullptr;  // HARRIS_SCORE: (response, record) scratch when a level exceeds LDS
    float* d_lvlResp = nullptr;   // HARRIS_SCORE: response of every kept keypoint
    float harrisScale4 = 0.f;
    int* d_rtab = nullptr;
    CellGeom* d_cells = nullptr;
    // per-stage HIP-event timing (orb_profile_*): stage k brackets its kernel(s) on the launch stream
    static constexpr int kStages = 5;
    // phases run by orb_extract_batch_device (the other entry points always run both):
    // bit 0 = pyramid (stages 0-1), bit 1 = detection, selection and descriptors (stages 2-4,
    // reading the pyramid bit 0 left in the workspace)
    unsigned phaseMask = 3u;
    bool pyrLegacy = false;        // orb_debug_set_pyramid_path(1): per-level launches at every batch size
    bool pyrStreamAlways = false;  // orb_debug_set_pyramid_path(2): k_pyr_stream at every batch size
    bool prof = false;
    unsigned profMask = 0;           // stages that record events (bit k = stage k)
    std::vector<hipEvent_t> evPool;  // 2 per stage per launch, recycled after each read
    std::vector<std::pair<int, int>> evPending;  // (stage, index of the start event)
    double stageMs[kStages] = {};
    long long stageLaunches[kStages] = {};
    int evNext = 0;
    // staging for host-buffer entry points
    uint8_t* d_img = nullptr;
    uint8_t* d_imgColor = nullptr;  // orb_extract_color's interleaved frame
    size_t imgColorCap = 0;
    // one device block: counts (maxBatch, padded to 256 B) | keypoints | descriptors, so a
    // single-frame download of the count and frame 0's keypoints is one contiguous copy
    uint8_t* d_out = nullptr;
    orb_keypoint_t* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_counts = nullptr;
    size_t countsPad = 0;
    // pinned host staging of the single-frame host entry points (orb_extract, orb_extract_color):
    // frame (W x H x up to 4 channels) | count + keypoints | descriptors, mirroring d_out, so the
    // uploads and downloads are DMA from page-locked memory and nothing is allocated per call
    uint8_t* h_pin = nullptr;
    size_t pinImg = 0;

    void free_events() {
        for (auto e : evPool) hipEventDestroy(e);
        evPool.clear();
        evPending.clear();
        evNext = 0;
    }

    void free_ws() {
        hipFree(d_pyr);
        hipFree(d_tiles);
        hipFree(d_cand);
        hipFree(d_cellCount);
        hipFree(d_cand2);
        hipFree(d_lvl);
        hipFree(d_lvlCount);
        hipFree(d_lvlInfo);
        hipFree(d_selDone);
        hipFree(d_slotLvl);
        hipFree(d_candH);
        hipFree(d_lvlResp);
        hipFree(d_rtab);
        hipFree(d_cells);
        hipFree(d_img);
        hipFree(d_imgColor);
        hipFree(d_out);
        hipFree(d_scol);
        hipFree(d_srows);
        hipFree(d_slv);
        hipFree(d_srounds);
        if (h_pin) (void)hipHostFree(h_pin);
        d_scol = nullptr;
        d_srows = nullptr;
        d_slv = nullptr;
        d_srounds = nullptr;
        streamOk = false;
        d_pyr = nullptr;
        d_tiles = nullptr;
        nTiles = 0;
        d_cand = nullptr;
        d_cellCount = nullptr;
        d_cand2 = nullptr;
        d_lvl = nullptr;
        d_lvlCount = nullptr;
        d_lvlInfo = nullptr;
        d_selDone = nullptr;
        d_slotLvl = nullptr;
        d_candH = nullptr;
        d_lvlResp = nullptr;
        d_rtab = nullptr;
        d_cells = nullptr;
        d_img = nullptr;
        d_imgColor = nullptr;
        imgColorCap = 0;
        d_out = nullptr;
        d_kps = nullptr;
        d_desc = nullptr;
        d_counts = nullptr;
        h_pin = nullptr;
        pinImg = 0;
        W = H = 0;
        pyrBatch = 0;
    }

    // ORBextractor ctor arithmetic (ORBextractor.cc:462-510)
    void init_params() {
        mvScaleFactor.assign(nlevels, 1.f);
        for (int i = 1; i < nlevels; ++i) mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
        float invScaleFactor = (float)(1.0f / scaleFactor);
        mvInvScaleFactor.assign(nlevels, 1.f);
        for (int i = 1; i < nlevels; ++i) mvInvScaleFactor[i] = mvInvScaleFactor[i - 1] * invScaleFactor;
        nDesired.assign(nlevels, 0);
        float factor = (float)(1.0 / scaleFactor);
        float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
        int sum = 0;
        for (int l = 0; l < nlevels - 1; ++l) {
            nDesired[l] = cvRoundH(nd);
            sum += nDesired[l];
            nd *= factor;
        }
        nDesired[nlevels - 1] = std::max(nfeatures - sum, 0);
        kpCap = 0;
        for (int n : nDesired) kpCap += n;
        int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
        for (int v = 0; v <= vmax; ++v) umax[v] = cvRoundH(std::sqrt(225.0 - v * v));
        for (int v = 15, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    // Per-frame-size geometry: level sizes, cell grids, resize tables, workspace.
    int build_geometry(int w0, int h0) {
        free_ws();
        Geom G{};
        G.L = nlevels;
        G.fastTh = std::min(std::max(fastTh, 0), 255);
        G.fastCl = fastCl;
        G.scoreType = scoreType;
        int k7[7];
        gaussian_taps7(k7);
        for (int i = 0; i < 4; ++i) G.taps[i] = k7[3 + i];
        if (G.taps[0] != 55 || G.taps[1] != 49 || G.taps[2] != 34 || G.taps[3] != 18)
            return set_err(ORB_EINVAL, "Gaussian taps differ from the kernel's constants (c_rowB, GP_*)");
        for (int v = 0; v < 16; ++v) G.umax[v] = umax[v];
        G.umaxNib = 0;
        for (int v = 0; v < 16; ++v) G.umaxNib |= (unsigned long long)umax[v] << (4 * v);
        std::vector<CellGeom> cl;
        cellLds = 0;
        std::vector<int> rt;
        long long pyrBytes = 0;
        int cand = 0, kpBase = 0;
        for (int l = 0; l < nlevels; ++l) {
            LevelGeom& lg = G.lv[l];
            float sc = mvInvScaleFactor[l];
            lg.w = cvRoundH((float)w0 * sc);
            lg.h = cvRoundH((float)h0 * sc);
            if (lg.w < 1 || lg.h < 1 || lg.w >= 4096 || lg.h >= 4096)
                return set_err(ORB_ENOTSUP, "level size out of the supported range [1, 4095]");
            lg.pitch = (lg.w + 2 * orbdev::EDGE + 15) & ~15;
            lg.ph = lg.h + 2 * orbdev::EDGE;
            lg.fstride = (long long)lg.pitch * lg.ph;
            lg.base = pyrBytes;
            pyrBytes += lg.fstride * maxBatch;
            lg.scale = mvScaleFactor[l];
            lg.size = (float)(int)(31 * mvScaleFactor[l]);
            lg.xsimd_blur = (lg.w / 4) * 4;
            lg.nDesired = nDesired[l];
            lg.kpBase = kpBase;
            kpBase += nDesired[l];
        }
        // cell grid (ORBextractor.cc:527-597)
        const float imageRatio = (float)G.lv[0].w / G.lv[0].h;
        for (int l = 0; l < nlevels; ++l) {
            LevelGeom& lg = G.lv[l];
            const int nD = nDesired[l];
            const int levelCols = (int)std::sqrt((float)nD / (5 * imageRatio));
            const int levelRows = (int)(imageRatio * levelCols);
            if (levelCols <= 0 || levelRows <= 0)
                return set_err(ORB_ENOTSUP, "level " + std::to_string(l) + " has an empty cell grid (the reference "
                                            "divides by zero here)");
            if (levelCols * levelRows > ORB_MAX_CELLS_PER_LEVEL)
                return set_err(ORB_ENOTSUP, "more than 256 cells per level");
            const int maxBX = lg.w - 16, maxBY = lg.h - 16;
            const int Wd = maxBX - 16, Hd = maxBY - 16;
            const int cellW = (int)std::ceil((float)Wd / levelCols);
            const int cellH = (int)std::ceil((float)Hd / levelRows);
            const int nCells = levelRows * levelCols;
            lg.rows = levelRows;
            lg.cols = levelCols;
            lg.nfc = (int)std::ceil((float)nD / nCells);
            lg.cellW = cellW;
            lg.cellH = cellH;
            lg.cellWm = (int)(uint32_t)((0x100000000ull + cellW - 1) / (uint64_t)cellW);
            lg.cellHm = (int)(uint32_t)((0x100000000ull + cellH - 1) / (uint64_t)cellH);
            lg.detX1 = std::max(maxBX, levelCols > 1 ? 16 + (levelCols - 1) * cellW : 0);
            lg.detY1 = std::max(maxBY, levelRows > 1 ? 16 + (levelRows - 1) * cellH : 0);
            // keypoints of non-last cells can sit past maxBorder (ORBextractor.cc:560-597); the
            // descriptor image must hold every sample they reach (|offset| <= 18)
            lg.ringX1 = std::max(lg.w + 3, lg.detX1 + 18);
            lg.ringY1 = std::max(lg.h + 3, lg.detY1 + 18);
            if (lg.ringX1 > lg.w + 12 || lg.ringY1 > lg.h + 12)
                return set_err(ORB_ENOTSUP, "cell grid too dense: rBRIEF samples leave the 16-px padding");
            if (cellW <= 0 || cellH <= 0) return set_err(ORB_ENOTSUP, "empty cell size");
            lg.cell0 = (int)cl.size();
            std::vector<int> iniXCol(levelCols, 0);
            float hY = cellH + 6;
            for (int i = 0; i < levelRows; ++i) {
                const float iniY = 16 + i * cellH - 3;
                bool rowSkip = false;
                if (i == levelRows - 1) {
                    hY = maxBY + 3 - iniY;
                    if (hY <= 0) rowSkip = true;
                }
                float hX = cellW + 6;
                for (int j = 0; j < levelCols; ++j) {
                    CellGeom c{};
                    c.level = l;
                    float iniX;
                    if (rowSkip) {
                        c.skipped = 1;
                    } else {
                        if (i == 0) {
                            iniX = 16 + j * cellW - 3;
                            iniXCol[j] = (int)iniX;
                        } else {
                            iniX = iniXCol[j];
                        }
                        if (j == levelCols - 1) {
                            hX = maxBX + 3 - iniX;
                            if (hX <= 0) c.skipped = 1;
                        }
                        if (!c.skipped) {
                            c.x0 = (int)iniX;
                            c.y0 = (int)iniY;
                            c.hx = (int)(iniX + hX) - c.x0;
                            c.hy = (int)(iniY + hY) - c.y0;
                            if (c.x0 < 0 || c.y0 < 0 || c.x0 + c.hx > lg.w || c.y0 + c.hy > lg.h)
                                return set_err(ORB_ENOTSUP, "cell ROI outside the level (the reference asserts)");
                            int dw = c.hx - 6, dh = c.hy - 6;
                            c.cap = (dw > 0 && dh > 0) ? ((dw + 1) / 2) * ((dh + 1) / 2) : 0;
                            if (dw > 0 && dh > 0) cellLds = std::max(cellLds, rerun_lds(dw, dh));
                        }
                    }
                    cl.push_back(c);
                }
            }
            // uniform slot stride per level (k_fast computes a cell's slots arithmetically)
            int capMax = 0;
            for (size_t i = lg.cell0; i < cl.size(); ++i) capMax = std::max(capMax, cl[i].cap);
            lg.candBase = cand;
            lg.capMax = capMax;
            for (size_t i = lg.cell0; i < cl.size(); ++i) cl[i].candOff = cand + (int)(i - lg.cell0) * capMax;
            cand += (int)(cl.size() - lg.cell0) * capMax;
        }
        G.selCap = select_cap(w0, h0);
        listLds = (size_t)(scoreType == ORB_HARRIS_SCORE ? 4 : 2) * G.selCap * 4;
        selectLds = std::max(cellLds, listLds);
        if (selectLds > 150 * 1024) return set_err(ORB_ENOTSUP, "FAST cell larger than the LDS budget");
        // resize tables, l >= 1
        for (int l = 1; l < nlevels; ++l) {
            LevelGeom& lg = G.lv[l];
            const LevelGeom& ls = G.lv[l - 1];
            const int sw = ls.w, sh = ls.h, dw = lg.w, dh = lg.h;
            double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
            double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
            int isx = cvRoundH(scale_x), isy = cvRoundH(scale_y);
            if (std::abs(scale_x - isx) < 2.220446049250313e-16 && std::abs(scale_y - isy) < 2.220446049250313e-16 &&
                isx == 2 && isy == 2)
                return set_err(ORB_ENOTSUP, "exact 2x level step (OpenCV switches to INTER_AREA)");
            lg.rtab = (int)rt.size();
            std::vector<int> xofs(dw), alpha(dw), yofs(dh), beta(dh);
            int xmax = dw;
            for (int dx = 0; dx < dw; ++dx) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) fx = 0, sx = 0;
                if (sx + 1 >= sw) {
                    xmax = std::min(xmax, dx);
                    if (sx >= sw - 1) fx = 0, sx = sw - 1;
                }
                xofs[dx] = sx;
                short a0 = satS16(cvRoundH((1.f - fx) * 2048)), a1 = satS16(cvRoundH(fx * 2048));
                alpha[dx] = (int)(uint16_t)a0 | ((int)(uint16_t)a1 << 16);
            }
            for (int dy = 0; dy < dh; ++dy) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = (int)std::floor(fy);
                fy -= sy;
                yofs[dy] = sy;
                short b0 = satS16(cvRoundH((1.f - fy) * 2048)), b1 = satS16(cvRoundH(fy * 2048));
                beta[dy] = (int)(uint16_t)b0 | ((int)(uint16_t)b1 << 16);
            }
            for (int dx = 0; dx < dw; ++dx) {  // k_pyr_resize's no-saturation premise
                const int c0 = alpha[dx] & 0xFFFF, c1 = (alpha[dx] >> 16) & 0xFFFF;
                if ((short)c0 < 0 || (short)c1 < 0 || c0 + c1 > 2050)
                    return set_err(ORB_ENOTSUP, "resize coefficient outside [0, 2050]");
            }
            for (int dy = 0; dy < dh; ++dy) {
                const int c0 = beta[dy] & 0xFFFF, c1 = (beta[dy] >> 16) & 0xFFFF;
                if ((short)c0 < 0 || (short)c1 < 0 || c0 + c1 > 2050)
                    return set_err(ORB_ENOTSUP, "resize coefficient outside [0, 2050]");
            }
            int xs = 0;
            while (xs <= dw - 16) xs += 16;
            while (xs < dw - 4) xs += 4;
            lg.xs_resize = xs;
            lg.xmax = xmax;
            rt.insert(rt.end(), xofs.begin(), xofs.end());
            rt.insert(rt.end(), alpha.begin(), alpha.end());
            rt.insert(rt.end(), yofs.begin(), yofs.end());
            rt.insert(rt.end(), beta.begin(), beta.end());
            // source rectangle of every RZ_TW x TH tile of the padded level (k_pyr_resize), for
            // the two tile heights
            auto tiles = [&](int TH, int& off, size_t& ldsOut) {
                const int tx = (lg.pitch + RZ_TW - 1) / RZ_TW, ty = (lg.ph + TH - 1) / TH;
                off = (int)rt.size();
                size_t lds = 0;
                for (int y = 0; y < ty; ++y)
                    for (int x = 0; x < tx; ++x) {
                        int c0 = INT32_MAX, c1 = -1, r0 = INT32_MAX, r1 = -1;
                        for (int px = x * RZ_TW; px < std::min((x + 1) * RZ_TW, lg.pitch); ++px) {
                            const int lx = orbdev::reflect101(std::min(px, dw + 31) - 16, dw);
                            const int sx = xofs[lx];
                            const int sx1 = (lx < xmax && (alpha[lx] >> 16) != 0) ? sx + 1 : sx;
                            c0 = std::min(c0, sx);
                            c1 = std::max(c1, sx1);
                        }
                        for (int py = y * TH; py < std::min((y + 1) * TH, lg.ph); ++py) {
                            const int ly = orbdev::reflect101(py - 16, dh);
                            r0 = std::min(r0, std::min(std::max(yofs[ly], 0), sh - 1));
                            r1 = std::max(r1, std::min(std::max(yofs[ly] + 1, 0), sh - 1));
                        }
                        const int cs = c0 & ~15, units = ((c1 - cs) >> 4) + 1, nr = r1 - r0 + 1;
                        rt.push_back(cs);
                        rt.push_back(units);
                        rt.push_back(r0);
                        rt.push_back(nr);
                        lds = std::max(lds, (size_t)units * 16 * nr);
                    }
                ldsOut = lds;
            };
            tiles(RZ_TH, lg.rtile, resizeLds[l]);
            tiles(RZ_THS, lg.rtileS, resizeLdsS[l]);
            if (resizeLds[l] > 96 * 1024) return set_err(ORB_ENOTSUP, "scale factor too large for the resize tile");
        }
        // the fused small-level tail: the first level from which every later level's source
        // ROI (ping-pong A / B) plus the staged tables fit the CU's LDS
        resizeTail = nlevels;
        for (int l = 1; l + 1 < nlevels; ++l) {
            auto roi = [&](int k) { return k + 1 < nlevels ? (size_t)G.lv[k].w * G.lv[k].h : (size_t)0; };
            const size_t a = (roi(l) + 15) & ~(size_t)15, bsz = (roi(l + 1) + 15) & ~(size_t)15;
            const size_t need = a + bsz + (size_t)8 * (G.lv[l].w + G.lv[l].h);
            if (need <= (size_t)RT_LDS_MAX && KR_TAIL) {
                resizeTail = l;
                tailBufA = (int)a;
                tailBufB = (int)bsz;
                tailLds = need;
                break;
            }
        }
        G.nCells = (int)cl.size();
        G.candPerFrame = cand;
        G.kpCap = kpCap;
        {  // k_orient_desc's grid is ((kpCap + slots - 1) / slots, B): bid / gridDim.x by multiply-high
            const unsigned long long gx = (unsigned long long)(std::max(kpCap, 1) + OD_WAVES - 1) / OD_WAVES;
            // and its per-slot offsets are 32-bit: descriptor bytes of the whole batch < 2^32
            if ((unsigned long long)std::max(kpCap, 1) * (unsigned long long)maxBatch * 32ull >= (1ull << 32))
                return set_err(ORB_ENOTSUP, "max_batch x keypoint capacity too large (descriptor bytes >= 4 GiB)");
            G.odDivMagic = (uint32_t)(((1ull << 32) + gx - 1) / gx);
            if (gx * gx * (unsigned long long)maxBatch >= (1ull << 32))
                return set_err(ORB_ENOTSUP, "keypoint grid too large for k_orient_desc's block decode");
        }
        // workspace
        // + slack: k_orient_desc's 64-byte window rows and k_rerun's 16-B ROI units may over-read
        // the last row's pitch
        HIP_TRY(hipMalloc(&d_pyr, (size_t)pyrBytes + 256));
        // k_fast tiles over each level's detection region: the width split evenly into
        // ceil(width / 256) tiles of a multiple of 4 columns, as many rows as the LDS budgets
        // (staged tile, strength plane) and the 16-bit queue codes allow
        std::vector<FastTile> tl;
        auto rcp = [](int d) { return (uint32_t)((0x100000000ull + (uint64_t)d - 1) / (uint64_t)d); };
        for (int l = 0; l < nlevels; ++l) {
            const int detW = G.lv[l].detX1 - orbdev::EDGE;
            const int nx = (detW + FT_TW_MAX - 1) / FT_TW_MAX;
            int tw4 = std::max(2, ((detW + 3) / 4 + nx - 1) / nx);
#if KF_B64
            tw4 = (tw4 + 1) & ~1;  // tiles of a multiple of 8 columns: every x0 = 0 mod 8
#endif
            const int TW = 4 * tw4;
            for (int x0 = orbdev::EDGE; x0 < G.lv[l].detX1; x0 += TW) {
#if KF_B64
                // first staged byte at sx = 16 + (x0 mod 16) in {16, 24}: the compass groups' dword
                // pairs (sx - 8 + 8 kp) 8-B aligned, and 16 bytes left of the tile for the left pair
                const int sx = 16 + (x0 & 15);
#else
                const int sx = x0 - (((x0 + orbdev::EDGE - 8) & ~15) - orbdev::EDGE);
#endif
                const int sp = (sx + TW + 8 + 15) & ~15, spw = TW + 8;
                const int thMax = std::min({FT_IN_BYTES / sp - 8, FT_S_BYTES / spw - 2, 126, 4095 / (tw4 + 2) - 2});
                if (thMax < 1 || sp > 288) return set_err(ORB_EINVAL, "k_fast tile geometry");
                for (int y0 = orbdev::EDGE; y0 < G.lv[l].detY1; y0 += thMax) {
                    const int th = std::min(thMax, G.lv[l].detY1 - y0);
                    tl.push_back(FastTile{l, x0, y0, tw4, th, sp, sx, rcp(tw4 + 2), rcp(tw4), rcp(sp >> 4)});
                }
            }
        }
        HIP_TRY(hipMalloc(&d_tiles, tl.size() * sizeof(FastTile)));
        HIP_TRY(hipMemcpy(d_tiles, tl.data(), tl.size() * sizeof(FastTile), hipMemcpyHostToDevice));
        nTiles = (int)tl.size();

        HIP_TRY(hipMalloc(&d_cand, (size_t)std::max(cand, 1) * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_cellCount, (size_t)G.nCells * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_cand2, (size_t)std::max(cand, 1) * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_lvl, (size_t)std::max(kpCap, 1) * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_lvlCount, (size_t)nlevels * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_lvlInfo, (size_t)ORB_MAX_LEVELS * maxBatch * sizeof(int2)));
        HIP_TRY(hipMalloc(&d_selDone, (size_t)maxBatch * sizeof(int)));
        HIP_TRY(hipMemset(d_selDone, 0, (size_t)maxBatch * sizeof(int)));
        {
            std::vector<uint8_t> sl(((size_t)std::max(kpCap, 1) + 3) & ~(size_t)3, 0);
            for (int l = 0; l < nlevels; ++l)
                for (int k = 0; k < G.lv[l].nDesired; ++k) sl[(size_t)G.lv[l].kpBase + k] = (uint8_t)l;
            HIP_TRY(hipMalloc(&d_slotLvl, sl.size()));
            HIP_TRY(hipMemcpy(d_slotLvl, sl.data(), sl.size(), hipMemcpyHostToDevice));
        }
        if (scoreType == ORB_HARRIS_SCORE) {
            HIP_TRY(hipMalloc(&d_candH, (size_t)std::max(cand, 1) * maxBatch * 8));
            HIP_TRY(hipMalloc(&d_lvlResp, (size_t)std::max(kpCap, 1) * maxBatch * 4));
        }
        HIP_TRY(hipMalloc(&d_rtab, std::max<size_t>(rt.size(), 1) * 4));
        HIP_TRY(hipMalloc(&d_cells, cl.size() * sizeof(CellGeom)));
        if (!rt.empty()) HIP_TRY(hipMemcpy(d_rtab, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_cells, cl.data(), cl.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
        if (int r = build_stream_plan(G, rt)) return r;
        g = G;
        cells = std::move(cl);
        rtab = std::move(rt);
        W = w0;
        H = h0;
        return ORB_OK;
    }

    // k_pyr_stream's plan: the round schedule (greedy: level l computes every row whose source
    // rows of level l-1 are in its ring), the ring capacity of each level (max over rounds of
    // newest row written - oldest row read + 1), ring slots, per-row and per-quad tables.  K0
    // (level-0 rows per round) is the largest whose rings fit PS_LDS_TARGET.  Frames with a
    // level under 17 px (multiple reflections) or rings that never fit keep the per-level path.
    int build_stream_plan(const Geom& G, const std::vector<int>& rt) {
        streamOk = false;
        const int L = nlevels;
        if (L < 2) return ORB_OK;
        for (int l = 0; l < L; ++l)
            if (G.lv[l].w < 17 || G.lv[l].h < 17) return ORB_OK;
        const int u0 = (G.lv[0].w + 15) / 16;
        std::vector<std::vector<int>> s0(L), s1(L);
        for (int l = 1; l < L; ++l) {
            const LevelGeom& lg = G.lv[l];
            const int hs = G.lv[l - 1].h;
            const int* yofs = rt.data() + lg.rtab + 2 * lg.w;
            s0[l].resize(lg.h);
            s1[l].resize(lg.h);
            for (int dy = 0; dy < lg.h; ++dy) {
                s0[l][dy] = std::min(std::max(yofs[dy], 0), hs - 1);
                s1[l][dy] = std::min(std::max(yofs[dy] + 1, 0), hs - 1);
            }
        }
        auto ringPitch = [&](int l) { return (G.lv[l].w + 15) & ~15; };
        auto nqOf = [&](int l) { return l == 0 ? G.lv[0].pitch / 16 : G.lv[l].pitch / 4; };
        // column words (LDS-resident): one u32 per padded column of levels >= 1
        // sx | a1 << 12 | (a0 - 2047 + a1) << 24 | simd << 26 | live << 27
        std::vector<uint32_t> cw;
        std::vector<int> colQuad(L, 0);
        for (int l = 1; l < L; ++l) {
            const LevelGeom& lg = G.lv[l];
            const int* xofs = rt.data() + lg.rtab;
            const int* alpha = xofs + lg.w;
            colQuad[l] = (int)(cw.size() / 4);
            for (int px = 0; px < 4 * nqOf(l); ++px) {
                const int lx = orbdev::reflect101(std::min(px, lg.w + 2 * orbdev::EDGE - 1) - orbdev::EDGE, lg.w);
                const int sx = xofs[lx];
                const int a0 = lx < lg.xmax ? (alpha[lx] & 0xFFFF) : 2048;
                const int a1 = lx < lg.xmax ? ((alpha[lx] >> 16) & 0xFFFF) : 0;
                const int d = a0 - 2047 + a1;
                if (sx < 0 || sx > 0xFFF || a1 > 0xFFF || d < 0 || d > 3) return ORB_OK;  // not encodable
                uint32_t c = (uint32_t)sx | ((uint32_t)a1 << 12) | ((uint32_t)d << 24);
                if (lx < lg.xs_resize) c |= 1u << 26;
                if (px < lg.w + 2 * orbdev::EDGE) c |= 1u << 27;
                cw.push_back(c);
            }
        }
        const size_t colBytes = (cw.size() * 4 + 15) & ~(size_t)15;
        std::vector<uint32_t> rounds;
        std::vector<int> cap;
        std::vector<std::vector<int>> plan;  // per round: lo, cnt per level
        int K0 = 0, maxEnt = 0;
        size_t lds = 0;
        for (int k0 : {32, 24, 16, 12, 8, 6, 4, 2}) {
            if (k0 * u0 > PS_NPF * 64 * PS_LOADERS) continue;
            std::vector<int> next(L, 0), cp(L, 0);
            std::vector<std::vector<int>> pl;
            int me = 0;
            bool ok = true;
            for (int n = 0;; ++n) {
                bool done = true;
                for (int l = 0; l < L; ++l) done = done && next[l] >= G.lv[l].h;
                if (done) break;
                if (n > 65536) {
                    ok = false;
                    break;
                }
                std::vector<int> lo(L), cnt(L);
                lo[0] = next[0];
                cnt[0] = std::min(k0, G.lv[0].h - next[0]);
                const int avail0 = next[0] + cnt[0];
                for (int l = 1; l < L; ++l) {
                    const int srcAvail = l == 1 ? avail0 : next[l - 1];
                    int d = next[l];
                    while (d < G.lv[l].h && s1[l][d] < srcAvail) ++d;
                    lo[l] = next[l];
                    cnt[l] = d - next[l];
                }
                for (int l = 0; l + 1 < L; ++l) {
                    // level 0: the loaders store round n+1's rows during round n
                    const int newest = (l == 0 ? std::min(avail0 + k0, G.lv[0].h) : next[l] + cnt[l]) - 1;
                    int oldest = INT32_MAX;
                    if (l == 0 && cnt[0]) oldest = lo[0];
                    if (cnt[l + 1]) oldest = std::min(oldest, s0[l + 1][lo[l + 1]]);
                    if (oldest != INT32_MAX) cp[l] = std::max(cp[l], newest - oldest + 1);
                }
                std::vector<int> rec(2 * L);
                int ent = 0;
                for (int l = 0; l < L; ++l) {
                    rec[2 * l] = lo[l];
                    rec[2 * l + 1] = cnt[l];
                    ent += cnt[l];
                    next[l] += cnt[l];
                }
                me = std::max(me, ent);
                pl.push_back(std::move(rec));
            }
            if (!ok || me > PS_NPF * 64 * PS_LOADERS) continue;
            size_t bytes = 0;
            bool capOk = true;
            for (int l = 0; l + 1 < L; ++l) {
                cp[l] = std::min(std::max(cp[l], 1), G.lv[l].h);
                capOk = capOk && cp[l] <= 255;
                bytes += (size_t)cp[l] * ringPitch(l);
            }
            const int stride8 = (me + 1) & ~1;
            bytes += colBytes;
            if (capOk && bytes <= PS_LDS_TARGET) {
                K0 = k0;
                plan = std::move(pl);
                cap = std::move(cp);
                maxEnt = stride8;
                lds = bytes;
                break;
            }
        }
        if (!K0) return ORB_OK;
        std::vector<StreamLevel> lv(L);
        int ringOff = 0;
        for (int l = 0; l < L; ++l) {
            const LevelGeom& lg = G.lv[l];
            StreamLevel& s = lv[l];
            s.nq = nqOf(l);
            s.nqm = (uint32_t)((0x100000000ull + s.nq - 1) / (uint64_t)s.nq);
            s.ringPitch = ringPitch(l);
            s.ringOff = l + 1 < L ? ringOff : 0;
            if (l + 1 < L) ringOff += cap[l] * s.ringPitch;
            s.w = lg.w;
            s.h = lg.h;
            s.pitch = lg.pitch;
            s.base = lg.base;
            s.fstride = lg.fstride;
        }
        // waves per level: one each, then greedily to the level with the most work per wave
        // (level-0 units are copies: weighted 1/4), up to one wave per 64 column units
        if (L > PS_THREADS / 64 - PS_LOADERS) return ORB_OK;
        {
            std::vector<int> nw(L, 1);
            for (int left = PS_THREADS / 64 - PS_LOADERS - L; left > 0; --left) {
                int best = -1;
                double bw = 0;
                for (int l = 0; l < L; ++l) {
                    if (nw[l] * 64 >= lv[l].nq) continue;
                    const double wk = (double)lv[l].nq * G.lv[l].h * (l == 0 ? 0.25 : 1.0) / nw[l];
                    if (wk > bw) {
                        bw = wk;
                        best = l;
                    }
                }
                if (best < 0) break;
                ++nw[best];
            }
            int ws = PS_LOADERS;
            for (int l = 0; l < L; ++l) {
                lv[l].waveStart = ws;
                lv[l].nWaves = nw[l];
                ws += nw[l];
            }
        }
        const int colOff = ringOff;  // multiple of 16
        for (int l = 1; l < L; ++l) lv[l].colOff = colOff + 16 * colQuad[l];
        lv[0].colOff = 0;
        // rounds (L level words + the first entry) and the row entries in round order: per row
        // {source row 0, source row 1 (LDS addresses), b0 << 12, b1 << 12, own ring row (LDS
        //  address or ~0u), padded-row offset, top mirror offset, bottom mirror offset (~0u: none)}
        std::vector<uint32_t> ent;
        for (const auto& rec : plan) {
            int ne = 0;
            for (int l = 0; l < L; ++l) {
                if (rec[2 * l] > 0xFFF || rec[2 * l + 1] > 0x3F || ne > 0x3FFF) return ORB_OK;
                rounds.push_back((uint32_t)rec[2 * l] | ((uint32_t)rec[2 * l + 1] << 12) | ((uint32_t)ne << 18));
                ne += rec[2 * l + 1];
            }
            rounds.push_back((uint32_t)(ent.size() / 8));
            rounds.push_back((uint32_t)ne);
            for (int l = 0; l < L; ++l)
                for (int dy = rec[2 * l]; dy < rec[2 * l] + rec[2 * l + 1]; ++dy) {
                    const LevelGeom& lg = G.lv[l];
                    const uint32_t own =
                        l + 1 < L ? (uint32_t)(lv[l].ringOff + (dy % cap[l]) * lv[l].ringPitch) : 0xFFFFFFFFu;
                    const uint32_t main = (uint32_t)((dy + orbdev::EDGE) * lg.pitch);
                    const uint32_t top = dy >= 1 && dy <= orbdev::EDGE ? (uint32_t)((orbdev::EDGE - dy) * lg.pitch) : 0xFFFFFFFFu;
                    const uint32_t bot = dy >= lg.h - 17 && dy <= lg.h - 2 ? (uint32_t)((2 * lg.h + 14 - dy) * lg.pitch) : 0xFFFFFFFFu;
                    if (l == 0) {
                        ent.insert(ent.end(), {own, 0u, 0u, 0u, 0xFFFFFFFFu, main, top, bot});
                    } else {
                        const int cs = cap[l - 1];
                        const uint32_t beta = (uint32_t)rt[lg.rtab + 2 * lg.w + lg.h + dy];
                        const uint32_t a0 = (uint32_t)(lv[l - 1].ringOff + (s0[l][dy] % cs) * lv[l - 1].ringPitch);
                        const uint32_t a1 = (uint32_t)(lv[l - 1].ringOff + (s1[l][dy] % cs) * lv[l - 1].ringPitch);
                        ent.insert(ent.end(), {a0, a1, (beta & 0xFFFFu) << 12, (beta >> 16) << 12, own, main, top, bot});
                    }
                }
        }
        // the magic divisions are exact over every task index of every round
        for (int l = 0; l < L; ++l) {
            int maxCnt = 0;
            for (const auto& rec : plan) maxCnt = std::max(maxCnt, rec[2 * l + 1]);
            for (uint32_t i = 0; i < (uint32_t)(maxCnt * lv[l].nq); ++i)
                if ((uint32_t)(((uint64_t)i * lv[l].nqm) >> 32) != i / (uint32_t)lv[l].nq) return ORB_OK;
        }
        StreamGeom sg{};
        sg.L = L;
        sg.nRounds = (int)plan.size();
        sg.u0 = u0;
        sg.u0m = (uint32_t)((0x100000000ull + u0 - 1) / (uint64_t)u0);
        for (uint32_t i = 0; i < (uint32_t)(K0 * u0); ++i)
            if ((uint32_t)(((uint64_t)i * sg.u0m) >> 32) != i / (uint32_t)u0) return ORB_OK;
        sg.colWords = (int)cw.size();
        sg.colOff = colOff;
        sg.rowOff = colOff + (int)colBytes;
        sg.rowStride = maxEnt;
        sg.cap0 = cap[0];
        HIP_TRY(hipMalloc(&d_scol, std::max<size_t>(cw.size(), 1) * 4));
        HIP_TRY(hipMemcpy(d_scol, cw.data(), cw.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&d_srows, ent.size() * 4));
        HIP_TRY(hipMemcpy(d_srows, ent.data(), ent.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&d_slv, L * sizeof(StreamLevel)));
        HIP_TRY(hipMemcpy(d_slv, lv.data(), L * sizeof(StreamLevel), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&d_srounds, rounds.size() * 4));
        HIP_TRY(hipMemcpy(d_srounds, rounds.data(), rounds.size() * 4, hipMemcpyHostToDevice));
        sgeom = sg;
        streamLds = lds;
        streamK0 = K0;
        streamOk = true;
        return ORB_OK;
    }

    int ensure_staging() {
        if (d_img) return ORB_OK;
        HIP_TRY(hipMalloc(&d_img, (size_t)W * H * maxBatch));
        const size_t cap = (size_t)std::max(kpCap, 1);
        countsPad = ((size_t)maxBatch * 4 + 255) & ~(size_t)255;
        const size_t kpsBytes = ((cap * maxBatch * sizeof(orb_keypoint_t)) + 255) & ~(size_t)255;
        HIP_TRY(hipMalloc(&d_out, countsPad + kpsBytes + cap * maxBatch * 32));
        d_counts = (int*)d_out;
        d_kps = (orb_keypoint_t*)(d_out + countsPad);
        d_desc = d_out + countsPad + kpsBytes;
        return ORB_OK;
    }

    // single-frame pinned staging: [frame: pinImg][count + frame-0 keypoints: countsPad + kpCap*28][descriptors]
    int ensure_pinned(size_t frameBytes) {
        if (h_pin && frameBytes <= pinImg) return ORB_OK;
        if (h_pin) {
            HIP_TRY(hipStreamSynchronize(stream));  // the previous call's copies are complete anyway
            (void)hipHostFree(h_pin);
            h_pin = nullptr;
            pinImg = 0;
        }
        const size_t img = (std::max(frameBytes, (size_t)W * H * 4) + 255) & ~(size_t)255;
        const size_t cap = (size_t)std::max(kpCap, 1);
        HIP_TRY(hipHostMalloc((void**)&h_pin, img + countsPad + cap * (sizeof(orb_keypoint_t) + 32), 0));
        pinImg = img;
        return ORB_OK;
    }

    // host frame (rows at `stride`) -> pinned -> device at `dst` (tight rows of `row` bytes)
    int upload_frame(uint8_t* dst, const uint8_t* img, size_t row, int hgt, size_t stride) {
        if (int r = ensure_pinned(row * hgt)) return r;
        if (stride == row) {
            std::memcpy(h_pin, img, row * hgt);
        } else {
            for (int y = 0; y < hgt; ++y) std::memcpy(h_pin + row * y, img + stride * y, row);
        }
        HIP_TRY(hipMemcpyAsync(dst, h_pin, row * hgt, hipMemcpyHostToDevice, stream));
        return ORB_OK;
    }

    // frame 0's count, keypoints and descriptors -> the caller's buffers (one stream sync)
    int download_frame0(orb_keypoint_t* kps_out, int kps_cap, uint8_t* desc_out, int* n_out) {
        const size_t cap = (size_t)std::max(kpCap, 1);
        uint8_t* pk = h_pin + pinImg;
        uint8_t* pd = pk + countsPad + cap * sizeof(orb_keypoint_t);
        HIP_TRY(hipMemcpyAsync(pk, d_out, countsPad + cap * sizeof(orb_keypoint_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipMemcpyAsync(pd, d_desc, cap * 32, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        int n = 0;
        std::memcpy(&n, pk, 4);
        if (n > kps_cap) return set_err(ORB_ERANGE, "kps_cap smaller than the number of keypoints");
        std::memcpy(kps_out, pk + countsPad, (size_t)n * sizeof(orb_keypoint_t));
        std::memcpy(desc_out, pd, (size_t)n * 32);
        *n_out = n;
        return ORB_OK;
    }

    hipEvent_t next_event() {
        if (evNext == (int)evPool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            evPool.push_back(e);
        }
        return evPool[evNext++];
    }
    // stage_begin pushes one entry per bracketed stage; an entry whose events could not be
    // created is a sentinel (index -1) that stage_end and profile_collect skip
    void stage_begin(int stage, hipStream_t st) {
        if (!prof || !((profMask >> stage) & 1u)) return;
        int i = evNext;
        hipEvent_t a = next_event(), b = next_event();
        if (!a || !b || hipEventRecord(a, st) != hipSuccess) {
            evPending.push_back({stage, -1});
            return;
        }
        evPending.push_back({stage, i});
    }
    void stage_end(int stage, hipStream_t st) {
        if (!prof || !((profMask >> stage) & 1u) || evPending.empty()) return;
        const auto& pe = evPending.back();
        if (pe.first != stage || pe.second < 0) return;
        hipEventRecord(evPool[pe.second + 1], st);
    }
    int profile_collect() {
        for (auto& pe : evPending) {
            if (pe.second < 0) continue;
            HIP_TRY(hipEventSynchronize(evPool[pe.second + 1]));
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, evPool[pe.second], evPool[pe.second + 1]));
            stageMs[pe.first] += ms;
            stageLaunches[pe.first] += 1;
        }
        evPending.clear();
        evNext = 0;
        return ORB_OK;
    }

    // Every launch on this handle's workspace is ordered after the previous one, whatever
    // stream either ran on: an event recorded on the previous stream is waited on by `st`
    // (device-side; the host never blocks).
    int order_after_last(hipStream_t st) {
        if (lastValid && lastStream != st) {
            HIP_TRY(hipEventRecord(evOrder, lastStream));
            HIP_TRY(hipStreamWaitEvent(st, evOrder, 0));
        }
        lastStream = st;
        lastValid = true;
        return ORB_OK;
    }
    // The workspace is about to be re-allocated: drain every stream that may still use it.
    int drain() {
        HIP_TRY(hipStreamSynchronize(stream));
        if (lastValid) HIP_TRY(hipStreamSynchronize(lastStream));
        return ORB_OK;
    }

    int launch(int B, const uint8_t* d_imgs, int stride, long long fpitch, orb_keypoint_t* kps, uint8_t* desc,
               int* counts, hipStream_t st, int cn = 1, int rgb = 0, unsigned phases = 3u) {
        if (!(phases & 1u) && B > pyrBatch)
            return set_err(ORB_EINVAL, "phase 2 without a phase-1 pyramid of this geometry for these frames");
        if (int r = order_after_last(st)) return r;
        if (prof && evNext > 4096) {  // bound the pool between reads
            int r = profile_collect();
            if (r) return r;
        }
        bool countsZeroed = false;  // k_pyr_stream zeroed k_fast's cell counters
        if ((phases & 1u) && cn == 1 && streamOk && (B >= KR_STREAM_BATCH || pyrStreamAlways) && !pyrLegacy) {
            // the whole pyramid in one streaming pass per frame (stage 0; stage 1 is empty)
            stage_begin(0, st);
            StreamGeom sg = sgeom;
            const uintptr_t al = (uintptr_t)d_imgs | (uintptr_t)stride | (uintptr_t)fpitch;
            sg.align = (al & 15u) == 0 ? 16 : (al & 3u) == 0 ? 4 : 1;
#if ORB_ILP_SPLIT
            orb_ilp_pyr_stream(B, streamLds, st, d_imgs, stride, fpitch, d_pyr, (const uint32_t*)d_scol,
                               (const uint4*)d_srows, (const StreamLevel*)d_slv, (const uint32_t*)d_srounds, sg,
                               (phases & 2u) ? d_cellCount : (int*)nullptr, g.nCells);
#else
            hipLaunchKernelGGL(k_pyr_stream, dim3(B), dim3(PS_THREADS), streamLds, st, d_imgs, stride, fpitch, d_pyr,
                               (const uint32_t*)d_scol, (const uint4*)d_srows, (const StreamLevel*)d_slv,
                               (const uint32_t*)d_srounds, sg, (phases & 2u) ? d_cellCount : (int*)nullptr, g.nCells);
#endif
            countsZeroed = (phases & 2u) != 0;
            stage_end(0, st);
            pyrBatch = B;
        } else if (phases & 1u) {
        stage_begin(0, st);
        {
            const LevelGeom& lg = g.lv[0];
            dim3 grid((lg.pitch / 4 + 63) / 64, (lg.ph + 3) / 4, B);
            if (cn == 1)
                hipLaunchKernelGGL(k_pyr0, dim3(((lg.pitch >> 4) * lg.ph + 255) / 256, B), dim3(256), 0, st, d_imgs,
                                   stride, fpitch, d_pyr, g);
            else  // R2Y on the red channel, B2Y on the blue one
                hipLaunchKernelGGL(k_pyr0_color, grid, dim3(64, 4), 0, st, d_imgs, stride, fpitch, cn,
                                   rgb ? 4899 : 1868, rgb ? 1868 : 4899, d_pyr, g);
        }
        stage_end(0, st);
        stage_begin(1, st);
        // a few frames: one multi-workgroup launch per level (the tail kernel's one workgroup
        // per frame walks its levels serially, the latency floor of a single frame)
        const int tail = B < KR_TAIL_BATCH ? nlevels : resizeTail;
        for (int l = 1; l < tail; ++l) {
            const LevelGeom& lg = g.lv[l];
            if (B < KR_SHORT_BATCH) {
                dim3 grid((lg.pitch + RZ_TW - 1) / RZ_TW, (lg.ph + RZ_THS - 1) / RZ_THS, B);
                hipLaunchKernelGGL(k_pyr_resize<RZ_THS>, grid, dim3(256), resizeLdsS[l], st, d_pyr, d_rtab, g.lv[l],
                                   g.lv[l - 1]);
            } else {
                dim3 grid((lg.pitch + RZ_TW - 1) / RZ_TW, (lg.ph + RZ_TH - 1) / RZ_TH, B);
                hipLaunchKernelGGL(k_pyr_resize<RZ_TH>, grid, dim3(256), resizeLds[l], st, d_pyr, d_rtab, g.lv[l],
                                   g.lv[l - 1]);
            }
        }
        if (tail < nlevels)
            hipLaunchKernelGGL(k_pyr_resize_tail, dim3(B), dim3(RT_THREADS), tailLds, st, d_pyr, d_rtab, g, resizeTail,
                               tailBufA, tailBufB);
        stage_end(1, st);
        pyrBatch = B;
        }
        if (!(phases & 2u)) {
            HIP_TRY(hipGetLastError());
            return ORB_OK;
        }
        stage_begin(2, st);
        if (!countsZeroed) HIP_TRY(hipMemsetAsync(d_cellCount, 0, (size_t)g.nCells * B * 4, st));
#if ORB_ILP_SPLIT
        orb_ilp_fast(nTiles, B, st, d_pyr, g, d_tiles, d_cand, d_cellCount);
#else
        hipLaunchKernelGGL(k_fast, dim3(nTiles, B), dim3(256), 0, st, d_pyr, g, d_tiles, d_cand, d_cellCount);
#endif
        stage_end(2, st);
        stage_begin(3, st);
        // FAST(7) re-runs: spread over NWG workgroups per level first (k_rerun), or inside
        // k_select (one workgroup per level and frame, no extra launch).  With the compass
        // pre-filtered re-run, apart is faster at every measured size (B = 512, re-run + select:
        // 640x480 0.190 vs 0.239 ms inside; 1241x376 0.497 vs 0.696; 1280x720 0.864 vs 1.421).
        const bool sep = (B < KS_SEP_BATCH || (long long)W * H > KS_SEP_PIXELS) && cellLds;
        if (sep) {
            const int NWG = std::min(32, std::max(KR_NWG_MIN, 512 / (B * nlevels)));
            hipLaunchKernelGGL(k_rerun, dim3(B * NWG, nlevels), dim3(256), cellLds, st, d_pyr, d_cand, d_cellCount, g,
                               d_cells, NWG);
        }
        const dim3 sg(B, nlevels);
        if (scoreType == ORB_HARRIS_SCORE) {
            if (sep)
                hipLaunchKernelGGL((k_select<true, false>), sg, dim3(256), listLds, st, d_pyr, d_cand, d_cand2,
                                   d_cellCount, g, d_cells, d_lvl, d_lvlCount, d_candH, d_lvlResp, harrisScale4, d_selDone,
                                   d_lvlInfo, counts);
            else
                hipLaunchKernelGGL((k_select<true, true>), sg, dim3(256), selectLds, st, d_pyr, d_cand, d_cand2,
                                   d_cellCount, g, d_cells, d_lvl, d_lvlCount, d_candH, d_lvlResp, harrisScale4, d_selDone,
                                   d_lvlInfo, counts);
        } else {
            if (sep)
                hipLaunchKernelGGL((k_select<false, false>), sg, dim3(256), listLds, st, d_pyr, d_cand, d_cand2,
                                   d_cellCount, g, d_cells, d_lvl, d_lvlCount, (uint64_t*)nullptr, (float*)nullptr, 0.f,
                                   d_selDone, d_lvlInfo, counts);
            else
                hipLaunchKernelGGL((k_select<false, true>), sg, dim3(256), selectLds, st, d_pyr, d_cand, d_cand2,
                                   d_cellCount, g, d_cells, d_lvl, d_lvlCount, (uint64_t*)nullptr, (float*)nullptr, 0.f,
                                   d_selDone, d_lvlInfo, counts);
        }
        // (the frames' per-level output offsets and totals: written by each frame's last k_select
        // workgroup, select_frame_done)
        if (hipError_t e = hipGetLastError(); e != hipSuccess) {
            // a k_select launch that did not run to completion leaves selDone[b] counting: clear it,
            // or the next extraction on this handle would take its frames' counts from stale levels
            (void)hipMemsetAsync(d_selDone, 0, (size_t)maxBatch * sizeof(int), st);
            return set_err(ORB_EDEVICE, std::string("k_select launch: ") + hipGetErrorString(e));
        }
        stage_end(3, st);
        stage_begin(4, st);
        dim3 gd((std::max(kpCap, 1) + OD_WAVES - 1) / OD_WAVES, B);
        hipLaunchKernelGGL(k_orient_desc, gd, dim3(64 * OD_WAVES), 0, st, d_pyr, g, d_lvl, d_slotLvl, d_lvlInfo, kps,
                           desc, (const float*)d_lvlResp);
        stage_end(4, st);
        HIP_TRY(hipGetLastError());
        return ORB_OK;
    }
};

static int upload_pattern(int device) {
    static bool uploaded[64] = {};
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (device >= 0 && device < 64 && uploaded[device]) return ORB_OK;
    float pf[1024];  // pair-major: point 8 l + q at pair 64 q + l (c_patternf)
    for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 8; ++q)
            for (int c = 0; c < 2; ++c) pf[2 * (64 * q + l) + c] = (float)kOrbPattern31[2 * (8 * l + q) + c];
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_patternf), pf, sizeof(pf)));
    {  // IC disc masks per alignment (umax of ORBextractor.cc:495-510, HALF_PATCH_SIZE 15)
        int um[16];
        const int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
        for (int v = 0; v <= vmax; ++v) um[v] = (int)lrint(std::sqrt(225.0 - v * v));
        for (int v = 15, v0 = 0; v >= vmin; --v) {
            while (um[v0] == um[v0 + 1]) ++v0;
            um[v] = v0;
            ++v0;
        }
        uint32_t off[320], c10[4 * 320] = {}, c01[4 * 320] = {};
        for (int n = 0; n < 320; ++n) off[n] = (uint32_t)(OD_WP * (n / 9) + 4 * (n % 9));
        for (int sh = 0; sh < 4; ++sh)
            for (int n = 0; n < 31 * 9; ++n) {
                const int r = n / 9, c = n % 9, v = std::abs(r - 15);
                uint32_t w10 = 0, w01 = 0;
                for (int i = 0; i < 4; ++i) {
                    const int u = 4 * c + i - sh - 15;
                    if (std::abs(u) <= um[v]) {
                        w10 |= (uint32_t)(uint8_t)(int8_t)u << (8 * i);
                        w01 |= (uint32_t)(uint8_t)(int8_t)(r - 15) << (8 * i);
                    }
                }
                c10[320 * sh + n] = w10;
                c01[320 * sh + n] = w01;
            }
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_icoff), off, sizeof(off)));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_ic10), c10, sizeof(c10)));
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_ic01), c01, sizeof(c01)));
    }
    {  // banded 7-tap row-pass matrix (GaussianBlur 7x7 sigma 2 fixed-point taps) + the bias rows
        static const int8_t tap[7] = {18, 34, 49, 55, 49, 34, 18};
        uint8_t bf[4 * 64 * 16];
        for (int t = 0; t < 4; ++t)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 16; ++j) {
                    const int k = 16 * (l >> 4) + j, n = 16 * t + (l & 15);
                    int8_t v = (k - n >= 0 && k - n <= 6) ? tap[k - n] : 0;
                    if (k >= 61) v = k == 63 ? 58 : 127;  // 127*127 + 127*127 + 11*58 = 128 * 257
                    bf[(t * 64 + l) * 16 + j] = (uint8_t)v;
                }
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_rowB), bf, sizeof(bf)));
        // OD_SB column-pass fragments (f16 bit patterns)
        uint16_t ca[3 * 64 * 8];
        for (int v = 0; v < 3; ++v)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int h = l >> 4, o = l & 15, ro = 4 * h + (j & 3);
                    const int d = (v == 0 ? 0 : v == 1 ? 16 : 12) + ro - o;
                    int wgt = (d >= 0 && d <= 6) ? tap[d] : 0;
                    if (v == 2 && ro < 4) wgt = 0;  // rows 28 .. 31: the block's other tile holds them
                    if (j >= 4) wgt *= 256;
                    // a positive integer < 2^14 as f16: exponent e = floor(log2), 10-bit mantissa
                    uint16_t hbits = 0;
                    if (wgt) {
                        int e = 0;
                        while ((wgt >> (e + 1)) != 0) ++e;
                        hbits = (uint16_t)(((e + 15) << 10) | (((wgt << 10) >> e) & 0x3FF));
                    }
                    ca[(v * 64 + l) * 8 + j] = hbits;
                }
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_colA), ca, sizeof(ca)));
    }
    if (device >= 0 && device < 64) uploaded[device] = true;
    return ORB_OK;
}

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

const char* orb_last_error(void) { return g_last_error.c_str(); }

const char* orb_version(void) { return "orb_hip gfx950 " __DATE__; }

int orb_extractor_create(int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th, int device,
                         int max_batch, orb_extractor_t** out) {
    if (!out) return set_err(ORB_EINVAL, "out is NULL");
    *out = nullptr;
    if (nfeatures <= 0 || nlevels <= 0 || nlevels > ORB_MAX_LEVELS || !(scale_factor > 1.0f) || max_batch <= 0)
        return set_err(ORB_EINVAL, "invalid extractor parameters");
    if (score_type != ORB_FAST_SCORE && score_type != ORB_HARRIS_SCORE)
        return set_err(ORB_EINVAL, "score_type must be HARRIS_SCORE(0) or FAST_SCORE(1)");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(ORB_EINVAL, "device ordinal out of range");
    HIP_TRY(hipSetDevice(device));
    int st = upload_pattern(device);
    if (st) return st;
    // k_select<true> (HARRIS_SCORE) stages (response, record) pairs: up to 96 KB of LDS
    hipFuncSetAttribute((const void*)k_select<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)k_select<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)k_select<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)k_select<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)k_rerun, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)k_pyr_resize_tail, hipFuncAttributeMaxDynamicSharedMemorySize, RT_LDS_MAX);
#if ORB_ILP_SPLIT
    orb_ilp_init();
#else
    hipFuncSetAttribute((const void*)k_pyr_stream, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
#endif
    orb_extractor* h = new orb_extractor();
    h->nfeatures = nfeatures;
    h->scaleFactor = scale_factor;
    h->nlevels = nlevels;
    h->scoreType = score_type;
    h->fastTh = fast_th;
    {  // HarrisResponses' scale (ORBextractor.cc:89-91), blockSize 7, in the reference's float steps
        float scale = (1 << 2) * 7 * 255.0f;
        scale = 1.0f / scale;
        h->harrisScale4 = scale * scale * scale * scale;
    }
    h->device = device;
    h->maxBatch = max_batch;
    h->init_params();
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->evOrder, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return set_err(ORB_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = h;
    return ORB_OK;
}

int orb_extractor_destroy(orb_extractor_t* h) {
    if (!h) return ORB_OK;
    hipSetDevice(h->device);
    (void)h->drain();
    h->free_ws();
    h->free_events();
    hipEventDestroy(h->evOrder);
    hipStreamDestroy(h->stream);
    delete h;
    return ORB_OK;
}

int orb_get_levels(const orb_extractor_t* h) { return h ? h->nlevels : ORB_EINVAL; }

float orb_get_scale_factor(const orb_extractor_t* h) { return h ? (float)h->scaleFactor : 0.f; }

int orb_get_max_keypoints(const orb_extractor_t* h) { return h ? h->kpCap : ORB_EINVAL; }

int orb_get_level_info(const orb_extractor_t* h, int* fpl, float* sf) {
    if (!h) return ORB_EINVAL;
    for (int l = 0; l < h->nlevels; ++l) {
        if (fpl) fpl[l] = h->nDesired[l];
        if (sf) sf[l] = h->mvScaleFactor[l];
    }
    return ORB_OK;
}

int orb_extract_batch_device(orb_extractor_t* h, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                             int64_t frame_pitch, orb_keypoint_t* d_kps, uint8_t* d_desc, int32_t* d_counts,
                             void* stream) {
    if (!h || B <= 0 || !d_imgs || !d_kps || !d_desc || !d_counts) return set_err(ORB_EINVAL, "bad arguments");
    if (B > h->maxBatch) return set_err(ORB_EINVAL, "B exceeds max_batch");
    if (w <= 0 || hgt <= 0 || stride < w || frame_pitch < (int64_t)stride * hgt)
        return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;  // NULL = the null stream, as everywhere in HIP
    if (w != h->W || hgt != h->H) {
        // the workspace is re-allocated: drain every stream that may still be using it
        if (int r = h->drain()) return r;
        int r = h->build_geometry(w, hgt);
        if (r) return r;
    }
    return h->launch(B, d_imgs, stride, frame_pitch, d_kps, d_desc, d_counts, st, 1, 0, h->phaseMask);
}

int orb_extract_batch(orb_extractor_t* h, int B, const uint8_t* imgs, int w, int hgt, int stride, int64_t frame_pitch,
                      orb_keypoint_t* kps_out, uint8_t* desc_out, int32_t* n_out) {
    if (!h || B <= 0 || !imgs || !kps_out || !desc_out || !n_out) return set_err(ORB_EINVAL, "bad arguments");
    if (B > h->maxBatch) return set_err(ORB_EINVAL, "B exceeds max_batch");
    if (w <= 0 || hgt <= 0 || stride < w || frame_pitch < (int64_t)stride * hgt)
        return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    if (w != h->W || hgt != h->H) {
        if (int r = h->drain()) return r;
        int st = h->build_geometry(w, hgt);
        if (st) return st;
    }
    // the copies below overwrite the staging a launch on another stream may still read
    if (int r = h->order_after_last(h->stream)) return r;
    int st = h->ensure_staging();
    if (st) return st;
    if (stride == w && frame_pitch == (int64_t)w * hgt) {  // tight frames: one linear copy
        HIP_TRY(hipMemcpyAsync(h->d_img, imgs, (size_t)B * w * hgt, hipMemcpyHostToDevice, h->stream));
    } else {
        for (int k = 0; k < B; ++k)
            HIP_TRY(hipMemcpy2DAsync(h->d_img + (size_t)k * w * hgt, w, imgs + (size_t)k * frame_pitch, stride, w,
                                     (size_t)hgt, hipMemcpyHostToDevice, h->stream));
    }
    st = h->launch(B, h->d_img, w, (long long)w * hgt, h->d_kps, h->d_desc, h->d_counts, h->stream);
    if (st) return st;
    HIP_TRY(hipMemcpyAsync(n_out, h->d_counts, (size_t)B * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemcpyAsync(kps_out, h->d_kps, (size_t)B * h->kpCap * sizeof(orb_keypoint_t), hipMemcpyDeviceToHost,
                           h->stream));
    HIP_TRY(hipMemcpyAsync(desc_out, h->d_desc, (size_t)B * h->kpCap * 32, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return ORB_OK;
}

int orb_extract(orb_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, orb_keypoint_t* kps_out,
                int kps_cap, uint8_t* desc_out, int* n_out) {
    if (!h || !n_out) return set_err(ORB_EINVAL, "bad arguments");
    if (w <= 0 || hgt <= 0) {  // _image.empty(): return, outputs untouched (ORBextractor.cc:721-722)
        *n_out = 0;
        return ORB_OK;
    }
    if (!img || !kps_out || !desc_out) return set_err(ORB_EINVAL, "bad arguments");
    if (stride < w) return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    if (w != h->W || hgt != h->H) {
        if (int r = h->drain()) return r;
        if (int r = h->build_geometry(w, hgt)) return r;
    }
    // the upload overwrites the staging a launch on another stream may still read
    if (int r = h->order_after_last(h->stream)) return r;
    if (int r = h->ensure_staging()) return r;
    if (int r = h->upload_frame(h->d_img, img, (size_t)w, hgt, (size_t)stride)) return r;
    if (int r = h->launch(1, h->d_img, w, (long long)w * hgt, h->d_kps, h->d_desc, h->d_counts, h->stream)) {
        (void)hipStreamSynchronize(h->stream);
        return r;
    }
    return h->download_frame0(kps_out, kps_cap, desc_out, n_out);
}

int orb_extract_batch_device_color(orb_extractor_t* h, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                                   int64_t frame_pitch, int channels, int rgb, orb_keypoint_t* d_kps, uint8_t* d_desc,
                                   int32_t* d_counts, void* stream) {
    if (!h || B <= 0 || !d_imgs || !d_kps || !d_desc || !d_counts) return set_err(ORB_EINVAL, "bad arguments");
    if (channels != 3 && channels != 4) return set_err(ORB_EINVAL, "channels must be 3 or 4");
    if (B > h->maxBatch) return set_err(ORB_EINVAL, "B exceeds max_batch");
    if (w <= 0 || hgt <= 0 || stride < w * channels || frame_pitch < (int64_t)stride * hgt)
        return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    if (w != h->W || hgt != h->H) {
        if (int r = h->drain()) return r;
        int r = h->build_geometry(w, hgt);
        if (r) return r;
    }
    return h->launch(B, d_imgs, stride, frame_pitch, d_kps, d_desc, d_counts, st, channels, rgb);
}

int orb_extract_color(orb_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, int channels, int rgb,
                      orb_keypoint_t* kps_out, int kps_cap, uint8_t* desc_out, int* n_out) {
    if (!h || !n_out) return set_err(ORB_EINVAL, "bad arguments");
    if (w <= 0 || hgt <= 0) {  // _image.empty(): return, outputs untouched (ORBextractor.cc:721-722)
        *n_out = 0;
        return ORB_OK;
    }
    if (!img || !kps_out || !desc_out) return set_err(ORB_EINVAL, "bad arguments");
    if (channels != 3 && channels != 4) return set_err(ORB_EINVAL, "channels must be 3 or 4");
    if (stride < w * channels) return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    if (w != h->W || hgt != h->H) {
        if (int r = h->drain()) return r;
        int r = h->build_geometry(w, hgt);
        if (r) return r;
    }
    if (int r = h->order_after_last(h->stream)) return r;
    int st = h->ensure_staging();
    if (st) return st;
    const size_t row = (size_t)w * channels;
    if (row * hgt > h->imgColorCap) {  // handle-owned, grow-only (the stream is ordered after every user)
        HIP_TRY(hipStreamSynchronize(h->stream));
        (void)hipFree(h->d_imgColor);
        h->d_imgColor = nullptr;
        h->imgColorCap = 0;
        HIP_TRY(hipMalloc(&h->d_imgColor, row * hgt));
        h->imgColorCap = row * hgt;
    }
    if (int r = h->upload_frame(h->d_imgColor, img, row, hgt, (size_t)stride)) return r;
    st = h->launch(1, h->d_imgColor, (int)row, (long long)(row * hgt), h->d_kps, h->d_desc, h->d_counts, h->stream,
                   channels, rgb);
    if (st) {
        (void)hipStreamSynchronize(h->stream);
        return st;
    }
    return h->download_frame0(kps_out, kps_cap, desc_out, n_out);
}

int orb_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        dist += __builtin_popcount(pa ^ pb);
    }
    return dist;
}

#ifndef MATCH_NMAX_NUM
#define MATCH_NMAX_NUM 9  // k_match_init's octave-0 capacity: NUM / 40 of the keypoint capacity
#endif
#ifndef MATCH_NMAX_MIN
#define MATCH_NMAX_MIN 256
#endif
static size_t match_lds_bytes(int cap, int nmax) {
    // F2 slots (desc 32 + state 8 + x,y,a,cell 16) + queries (q2i,qx,qy,angle 16 + top-8 32 +
    // cnt 4) + cap x (m12 4 + slot 2): nmax 1024 and cap 8192 fit (156 KB)
    return (size_t)nmax * (56 + 52) + (size_t)cap * 6 + 32;
}
static size_t match_big_lds_bytes(int cap, int nmax) { return (size_t)nmax * 8 + (size_t)cap * 6 + 16; }

// Global scratch of the large-capacity matcher body: one slot per pair, grow-only, one buffer per
// (device, stream) so launches on one stream reuse it in stream order and concurrent streams
// never share one.  Grown by a stream-ordered free + allocation on that stream; steady state:
// no allocator call.  Only the slots of pairs that overflow the LDS capacity are ever touched.
// The caller holds g_bigMu from the lookup until its launch is enqueued: two host threads
// sharing one stream (e.g. the null stream) then cannot interleave a grow (whose free is
// stream-ordered after the other thread's launch) between the other's lookup and launch.
static std::mutex g_bigMu;
static std::vector<std::pair<std::pair<int, hipStream_t>, std::pair<void*, size_t>>> g_big;
static int match_big_scratch_locked(hipStream_t st, size_t bytes, void** out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    for (auto& e : g_big)
        if (e.first.first == dev && e.first.second == st) {
            if (e.second.second < bytes) {
                HIP_TRY(hipFreeAsync(e.second.first, st));
                e.second = {nullptr, 0};
                HIP_TRY(hipMallocAsync(&e.second.first, bytes, st));
                e.second.second = bytes;
            }
            *out = e.second.first;
            return ORB_OK;
        }
    void* p = nullptr;
    HIP_TRY(hipMallocAsync(&p, bytes, st));
    g_big.push_back({{dev, st}, {p, bytes}});
    *out = p;
    return ORB_OK;
}

int orb_match_release_stream_scratch(void* stream) {
    hipStream_t st = (hipStream_t)stream;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_bigMu);
    for (size_t i = 0; i < g_big.size(); ++i)
        if (g_big[i].first.first == dev && g_big[i].first.second == st) {
            HIP_TRY(hipFreeAsync(g_big[i].second.first, st));  // after the stream's queued launches
            g_big.erase(g_big.begin() + (long)i);
            return ORB_OK;
        }
    return ORB_OK;
}

// A stream with every CU in its mask: the runtime gives a CU-masked stream a hardware queue of
// its own instead of sharing one of its GPU_MAX_HW_QUEUES round-robin (include/orb_abi.h).
int orb_stream_create_dedicated(void** out_stream) {
    if (!out_stream) return set_err(ORB_EINVAL, "bad arguments");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    int ncu = 0;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0xFFFFFFFFu);
    if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    hipStream_t st = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    *out_stream = (void*)st;
    return ORB_OK;
}

int orb_stream_destroy(void* stream) {
    if (!stream) return set_err(ORB_EINVAL, "bad arguments");
    orb_match_release_stream_scratch(stream);
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return ORB_OK;
}

// The batched launch; `done` / `doneSeq`: a host call's completion flag (P == 1), else null.
static int sfi_launch(const orb_keypoint_t* d_kps, const uint8_t* d_desc, const int32_t* d_counts, int cap, int P,
                      const int32_t* d_pair_f1, const int32_t* d_pair_f2, orb_frame_bounds_t bounds, float nnratio,
                      int check_ori, int window, float* d_prev_xy, int32_t* d_matches12, int32_t* d_nmatches,
                      void* stream, int* done, int doneSeq) {
    if (!d_kps || !d_desc || !d_counts || cap <= 0 || P < 0 || !d_pair_f1 || !d_pair_f2 || !d_matches12 ||
        !d_nmatches)
        return set_err(ORB_EINVAL, "bad arguments");
    if (((uintptr_t)d_desc & 15) != 0) return set_err(ORB_EINVAL, "descriptors must be 16-B aligned");
    if (P == 0) return ORB_OK;
    if (bounds.max_x <= bounds.min_x || bounds.max_y <= bounds.min_y) return set_err(ORB_EINVAL, "bad bounds");
    if (cap > MATCH_BIG_NMAX) return set_err(ORB_ENOTSUP, "more than 8192 keypoints per frame");
    // octave-0 keypoints per frame held in LDS by k_match_init.  The extractor keeps at most
    // mnFeaturesPerLevel[0] of them (0.217 nFeatures at scale 1.2, 8 levels), so when the pairs
    // fill the chip, 0.225 of the capacity covers its output and leaves room for two or more
    // work-groups per CU (640x480: 0.233 -> 0.129 ms for 511 pairs, 1241x376: 0.47 -> 0.26);
    // any frame beyond (another producer, another scale factor) is redone exactly by
    // the large-capacity body in the same workgroup.  Fewer pairs than CUs: one work-group per CU anyway, and the
    // full capacity spares the per-frame path the fallback scratch.
    const int capA = (cap + 3) & ~3;  // nmax a multiple of 4: k_match_init's LDS arrays 16-B aligned
    const int nmax = P < 256 ? std::min(capA, 1024)
                             : std::min({capA, 1024, std::max(MATCH_NMAX_MIN,
                                                             (int)(((long long)cap * MATCH_NMAX_NUM / 40 + 31) & ~31))});
    const int nmaxBig = std::min(cap, MATCH_BIG_NMAX);
    // the large-capacity body runs in the same workgroup: the dynamic LDS covers both
    size_t lds = std::max(match_lds_bytes(cap, nmax), cap > nmax ? match_big_lds_bytes(cap, nmaxBig) : 0);
    if (lds > 159 * 1024)  // 160 KB per CU minus the kernel's static LDS
        return set_err(ORB_ENOTSUP, "per-frame keypoint capacity too large for LDS");
    // the fixed-point phase 2 of the 16-wave launch: two acceptor lists (3 entries + count per
    // slot), decisions old / new and the rescan list per query, after the body's arrays
    int fixOff = 0;
    const size_t fixAt = (match_lds_bytes(cap, nmax) + 15) & ~(size_t)15;
    const size_t fixEnd = fixAt + (size_t)nmax * (2 * 16 + 8 + 2);
    const bool wide = P < KM_WIDE_PAIRS || KM_WIDE_ALL;  // 16-wave workgroups
    const int ntLaunch = wide ? 2 * KM_THREADS : KM_THREADS;
    if (KM_FIX && (wide || KM_FIX_BATCH) && nmax <= ntLaunch && fixEnd <= 158 * 1024) {
        fixOff = (int)fixAt;
        lds = std::max(lds, fixEnd);
    }
    static std::once_flag attrOnce;
    std::call_once(attrOnce, [] {
        (void)hipFuncSetAttribute((const void*)k_match_init<KM_THREADS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  159 * 1024);
        (void)hipFuncSetAttribute((const void*)k_match_init<2 * KM_THREADS>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024);
        (void)hipGetLastError();  // an unsupported attribute value must not surface as the launch's error
    });
    MatchGeom mg{bounds.min_x, bounds.max_x, bounds.min_y, bounds.max_y,
                 static_cast<float>(64) / static_cast<float>(bounds.max_x - bounds.min_x),
                 static_cast<float>(48) / static_cast<float>(bounds.max_y - bounds.min_y)};
    MatchArgs A{d_kps,      d_desc,    d_counts,     cap,       nmax,   d_pair_f1,         d_pair_f2,
                mg,         nnratio,   check_ori,    (float)window, d_prev_xy, d_matches12, d_nmatches,
                P,          P == 1 ? done : nullptr, doneSeq, fixOff};
    hipStream_t st = (hipStream_t)stream;
    void* big = nullptr;
    std::unique_lock<std::mutex> lk(g_bigMu, std::defer_lock);
    if (cap > nmax) {  // a pair may overflow the LDS capacity: its slot of the large-capacity scratch
        lk.lock();     // held until the launch that uses it is enqueued
        if (int r = match_big_scratch_locked(st, match_big_slot_bytes(cap, nmaxBig) * (size_t)P, &big)) return r;
    }
    if (wide)
        hipLaunchKernelGGL(k_match_init<2 * KM_THREADS>, dim3(P), dim3(2 * KM_THREADS), lds, st, A, (uint8_t*)big, nmaxBig);
    else
        hipLaunchKernelGGL(k_match_init<KM_THREADS>, dim3(P), dim3(KM_THREADS), lds, st, A, (uint8_t*)big, nmaxBig);
    HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orb_search_for_initialization_batch_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                               const int32_t* d_counts, int cap, int P, const int32_t* d_pair_f1,
                                               const int32_t* d_pair_f2, orb_frame_bounds_t bounds, float nnratio,
                                               int check_ori, int window, float* d_prev_xy, int32_t* d_matches12,
                                               int32_t* d_nmatches, void* stream) {
    return sfi_launch(d_kps, d_desc, d_counts, cap, P, d_pair_f1, d_pair_f2, bounds, nnratio, check_ori, window,
                      d_prev_xy, d_matches12, d_nmatches, stream, nullptr, 0);
}

int orb_search_for_initialization(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1, const orb_keypoint_t* kps2,
                                  const uint8_t* desc2, int n2, orb_frame_bounds_t bounds, float nnratio,
                                  int check_ori, int window, float* prev_xy, int32_t* matches12, int* n_matches) {
    if (n1 < 0 || n2 < 0 || !n_matches || (n1 > 0 && (!kps1 || !desc1 || !prev_xy || !matches12)) ||
        (n2 > 0 && (!kps2 || !desc2)))
        return set_err(ORB_EINVAL, "bad arguments");
    for (int i = 0; i < n1; ++i)
        if (kps1[i].octave < 0) return set_err(ORB_EINVAL, "negative octave in F1");
    *n_matches = 0;
    if (n1 == 0) return ORB_OK;
    const int cap = std::max(std::max(n1, n2), 1);
    if (n1 > MATCH_BIG_NMAX || n2 > MATCH_BIG_NMAX) return set_err(ORB_ENOTSUP, "more than 8192 keypoints in a frame");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    // the calling thread's context: grow-only pinned staging, its own stream (no per-call
    // allocation, no device-wide synchronisation).  The kernel reads its inputs from the pinned
    // staging and writes vnMatches12 / vbPrevMatched / nmatches back into it: no H2D or D2H
    // command (one SearchForInitialization call 64 -> 57 us at 640x480 / 1000 kp,
    // scripts/sfi_breakdown.cpp)
    OrbHostCtx* C = orb_internal_thread_ctx(dev);
    if (!C) return set_err(ORB_EINVAL, "device ordinal out of range");
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t oK = 0, oD = oK + al((size_t)2 * cap * sizeof(orb_keypoint_t)), oC = oD + al((size_t)2 * cap * 32),
                 oP = oC + al(6 * sizeof(int)), oM = oP + al((size_t)cap * 8), oF = oM + al((size_t)cap * 4 + 4),
                 total = oF + 256;
    if (int r = C->reserve(0, total)) return r;
    uint8_t* hs = C->pinned;
    std::memcpy(hs + oK, kps1, (size_t)n1 * sizeof(orb_keypoint_t));
    if (n2) std::memcpy(hs + oK + (size_t)cap * sizeof(orb_keypoint_t), kps2, (size_t)n2 * sizeof(orb_keypoint_t));
    std::memcpy(hs + oD, desc1, (size_t)n1 * 32);
    if (n2) std::memcpy(hs + oD + (size_t)cap * 32, desc2, (size_t)n2 * 32);
    const int hostc[6] = {n1, n2, 0, 1, 0, 0};  // counts of frames 0/1, pair (0, 1)
    std::memcpy(hs + oC, hostc, sizeof(hostc));
    std::memcpy(hs + oP, prev_xy, (size_t)n1 * 8);
    hipStream_t s = C->stream;
    int* dc = (int*)(hs + oC);
    int* dm = (int*)(hs + oM);
    // completion: the kernel's last act is a system-scope release then a flag store into the
    // staging; the call spins on the flag (~1 us after the kernel's write, where a stream
    // synchronisation takes several) and synchronises the stream only when the flag does not
    // come (an error, or a kernel beyond the bound) -- the staging is then reused by the next call
    // only after the flag: the kernel writes nothing after it
    static thread_local int seq = 0;
    seq = seq == 0x7fffffff ? 1 : seq + 1;
    volatile int* flag = (volatile int*)(hs + oF);
    *flag = 0;
    int st = sfi_launch((const orb_keypoint_t*)(hs + oK), hs + oD, dc, cap, 1, dc + 2, dc + 3, bounds, nnratio, check_ori,
                        window, (float*)(hs + oP), dm, dm + cap, s, (int*)(hs + oF), seq);
    bool seen = false;
    if (st == ORB_OK) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0;; ++spin) {
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) {
                seen = true;
                break;
            }
            if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        }
    }
    const hipError_t e = seen ? hipSuccess : hipStreamSynchronize(s);
    if (st) return st;
    if (e != hipSuccess) return set_err(ORB_EDEVICE, std::string("match: ") + hipGetErrorString(e));
    int nm = 0;
    std::memcpy(&nm, hs + oM + (size_t)cap * 4, 4);
    if (nm < 0) return set_err(ORB_ENOTSUP, "more octave-0 keypoints than the matcher holds");
    std::memcpy(matches12, hs + oM, (size_t)n1 * 4);
    std::memcpy(prev_xy, hs + oP, (size_t)n1 * 8);
    *n_matches = nm;
    return ORB_OK;
}

static const char* kStageNames[] = {"k_pyr0", "k_pyr_resize", "k_fast", "k_select", "k_orient_desc"};

int orb_profile_enable(orb_extractor_t* h, int enable) {
    return orb_profile_enable_stages(h, enable ? (1u << orb_extractor::kStages) - 1u : 0u);
}

int orb_debug_set_pyramid_path(orb_extractor_t* h, int mode) {
    if (!h || mode < 0 || mode > 2) return set_err(ORB_EINVAL, "mode must be 0, 1 or 2");
    h->pyrLegacy = mode == 1;
    h->pyrStreamAlways = mode == 2;
    return ORB_OK;
}

int orb_debug_set_fast_corner_list(orb_extractor_t* h, int cap) {
    if (!h || cap < 0 || cap > FT_CL) return set_err(ORB_EINVAL, "cap must be in [0, 256]");
    h->fastCl = cap;
    h->g.fastCl = cap;
    return ORB_OK;
}

int orb_debug_pyramid_plan(const orb_extractor_t* h, int* rows_per_round, int* rounds, int* lds_bytes) {
    if (!h) return set_err(ORB_EINVAL, "bad handle");
    if (!h->streamOk) return 0;
    if (rows_per_round) *rows_per_round = h->streamK0;
    if (rounds) *rounds = h->sgeom.nRounds;
    if (lds_bytes) *lds_bytes = (int)h->streamLds;
    return 1;
}

int orb_extract_set_phases(orb_extractor_t* h, unsigned phase_mask) {
    if (!h) return set_err(ORB_EINVAL, "bad handle");
    if (phase_mask == 0u || (phase_mask & ~3u)) return set_err(ORB_EINVAL, "phase_mask must be 1, 2 or 3");
    h->phaseMask = phase_mask;
    return ORB_OK;
}

int orb_profile_enable_stages(orb_extractor_t* h, unsigned stage_mask) {
    if (!h) return set_err(ORB_EINVAL, "bad handle");
    HIP_TRY(hipSetDevice(h->device));
    int r = h->profile_collect();
    if (r) return r;
    h->profMask = stage_mask & ((1u << orb_extractor::kStages) - 1u);
    h->prof = h->profMask != 0;
    for (int k = 0; k < orb_extractor::kStages; ++k) {
        h->stageMs[k] = 0;
        h->stageLaunches[k] = 0;
    }
    return ORB_OK;
}

int orb_profile_read(orb_extractor_t* h, double* stage_ms, int64_t* stage_launches, int nstages) {
    if (!h || nstages < 0) return set_err(ORB_EINVAL, "bad arguments");
    HIP_TRY(hipSetDevice(h->device));
    int r = h->profile_collect();
    if (r) return r;
    for (int k = 0; k < nstages && k < orb_extractor::kStages; ++k) {
        if (stage_ms) stage_ms[k] = h->stageMs[k];
        if (stage_launches) stage_launches[k] = h->stageLaunches[k];
    }
    return orb_extractor::kStages;
}

const char* orb_profile_stage_name(int i) {
    return (i >= 0 && i < orb_extractor::kStages) ? kStageNames[i] : "";
}

// ---- debug / test hooks (no device work) ------------------------------------------------
// Host instantiation of the device nth_element replay, for CPU unit tests.
int orb_debug_nth_element_u32(uint32_t* a, int n, int nth) {
    ScoreGreater comp;
    orbsel::nth_element(a, nth, n, comp);
    return ORB_OK;
}

}  // extern "C"

__global__ void __launch_bounds__(64) k_debug_nth_wave(uint32_t* a, int n, int nth) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_a[];
    uint16_t* Lp = (uint16_t*)(s_a + n);
    for (int i = threadIdx.x; i < n; i += 64) s_a[i] = a[i];
    __syncthreads();
    ScoreGreater comp;
    orbsel::nth_element_wave(s_a, nth, n, comp, Lp, Lp + n, (int)threadIdx.x);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 64) a[i] = s_a[i];
}

extern "C" {

int orb_debug_nth_element_wave_u32(uint32_t* a, int n, int nth, int device) {
    if (!a || n < 0 || n > 8192 || nth < 0 || nth > n) return set_err(ORB_EINVAL, "bad arguments");
    if (n == 0) return ORB_OK;
    HIP_TRY(hipSetDevice(device));
    uint32_t* d = nullptr;
    HIP_TRY(hipMalloc(&d, (size_t)n * 4));
    hipError_t e = hipMemcpy(d, a, (size_t)n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        (void)hipFuncSetAttribute((const void*)k_debug_nth_wave, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        hipLaunchKernelGGL(k_debug_nth_wave, dim3(1), dim3(64), (size_t)n * 8, 0, d, n, nth);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(a, d, (size_t)n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(ORB_EDEVICE, std::string("nth_element_wave: ") + hipGetErrorString(e));
    return ORB_OK;
}

// Download a padded pyramid level of frame `b` (after the last batch) into `out`
// ((w+32) x (h+32) bytes, tightly packed).  Synchronises the handle's stream.
int orb_debug_level_image(orb_extractor_t* h, int b, int l, uint8_t* out, int* w, int* hgt) {
    if (!h || l < 0 || l >= h->nlevels || !h->d_pyr) return set_err(ORB_EINVAL, "bad arguments");
    const LevelGeom& lg = h->g.lv[l];
    if (w) *w = lg.w;
    if (hgt) *hgt = lg.h;
    if (!out) return ORB_OK;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy2D(out, lg.w + 32, h->d_pyr + lg.base + (long long)b * lg.fstride, lg.pitch, lg.w + 32, lg.ph,
                        hipMemcpyDeviceToHost));
    return ORB_OK;
}

// Descriptor image of level l, frame b (blurred ROI + raw padding), padded layout, computed by
// k_debug_desc_image with k_orient_desc's rounding (the product never materialises it).
int orb_debug_blur_image(orb_extractor_t* h, int b, int l, uint8_t* out) {
    if (!h || l < 0 || l >= h->nlevels || !h->d_pyr || !out) return set_err(ORB_EINVAL, "bad arguments");
    const LevelGeom& lg = h->g.lv[l];
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    const size_t n = (size_t)(lg.w + 32) * (lg.h + 32);
    uint8_t* d = nullptr;
    HIP_TRY(hipMalloc(&d, n));
    hipLaunchKernelGGL(k_debug_desc_image, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, h->d_pyr, lg, b, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(out, d, n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(ORB_EDEVICE, std::string("debug descriptor image: ") + hipGetErrorString(e));
    return ORB_OK;
}

#if PS_TIMING
extern "C" int orb_debug_ps_timing(unsigned long long* out6) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out6, HIP_SYMBOL(g_pstime), 32 * sizeof(unsigned long long)));
    unsigned long long z[32] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pstime), z, sizeof(z)));
    return ORB_OK;
}
#endif
#if KM_TIMING
// experiment builds: k_match_init's per-phase s_memrealtime (100 MHz) sums
// {phase 0, rank, phase 1, phase 2, phase 3, pairs, queries, candidates}
extern "C" int orb_debug_km_timing(unsigned long long* out8) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_kmtime), 8 * sizeof(unsigned long long)));
    unsigned long long z[8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kmtime), z, sizeof(z)));
    return ORB_OK;
}
#endif
// Per-cell FAST counts (after fallback) of frame `b`, level `l`, row-major cells.
#if KR_TIMING
// experiment builds: k_rerun's per-level phase sums, [level][8] (see cell_fast_rerun)
int orb_debug_kr_timing(unsigned long long* out) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_krtime), sizeof(g_krtime)));
    static unsigned long long z[ORB_MAX_LEVELS][8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_krtime), z, sizeof(z)));
    return ORB_OK;
}
#endif
#if KS_TIMING
// experiment builds: k_select's per-level phase sums, [level][8] (see the kernel)
int orb_debug_ks_timing(unsigned long long* out) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kstime), sizeof(g_kstime)));
    static unsigned long long z[ORB_MAX_LEVELS][8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kstime), z, sizeof(z)));
    return ORB_OK;
}
#endif
#if KF_TIMING
// experiment builds: k_fast's per-phase s_memtime sums {stage, rows, drain, barrier, nms, waves}
int orb_debug_kf_timing(unsigned long long* out6) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out6, HIP_SYMBOL(g_kftime), 6 * sizeof(unsigned long long)));
    unsigned long long z[8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_kftime), z, sizeof(z)));
    return ORB_OK;
}
#endif
int orb_debug_cell_counts(orb_extractor_t* h, int b, int l, int* counts, int cap) {
    if (!h || l < 0 || l >= h->nlevels || !h->d_cellCount) return set_err(ORB_EINVAL, "bad arguments");
    const LevelGeom& lg = h->g.lv[l];
    int n = lg.rows * lg.cols;
    if (n > cap) return ORB_ERANGE;
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(counts, h->d_cellCount + (long long)b * h->g.nCells + lg.cell0, (size_t)n * 4,
                      hipMemcpyDeviceToHost));
    return n;
}

}  // extern "C"
#endif  // ORB_TU_MAIN (host side)
