// orb_hip.hip — MI355X (gfx950) ORB front end: kernels + the C ABI of include/orb_abi.h.
//
// Pipeline for a batch of B same-size frames (all device-resident, one HIP stream):
//   k_pyr0        level 0 + reflect-101 padding          (ORBextractor.cc:814-815)
//   k_pyr_resize  level l from level l-1, fused padding   (ORBextractor.cc:800-807), l = 1..L-1
//   k_fast_cells  per-cell FAST(th) / FAST(7) + 3x3 NMS + raster-order compaction
//                                                          (ORBextractor.cc:560-614)
//   k_select      per (frame, level): quota redistribution, retainBest per cell, level
//                 retainBest — exact libstdc++ nth_element replay (ORBextractor.cc:622-701)
//   k_orient_desc per keypoint (one wave): IC angle on the raw level, rBRIEF on the
//                 7x7 sigma-2 blur evaluated at the sample points, keypoint record
//                                                          (ORBextractor.cc:124-194, 705-777)
//   k_match_init  per frame pair (one wave): SearchForInitialization (ORBmatcher.cc:598-713)
//
// Reference behaviour that lives in OpenCV 2.4 / libstdc++ / glibc is restated per
// SURVEY.md Appendix A; DESIGN.md lists every arithmetic rule and where it is pinned.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"
#include "nth_select.h"
#include "orb_device.h"
#include "pattern31.inc"

#define ORB_MAX_LEVELS 16
#define ORB_MAX_CELLS_PER_LEVEL 256
#define ORB_SELECT_LDS_CAP 6144  // level list kept in LDS when it fits (u32 entries)

// ======================================================================================
// error plumbing
// ======================================================================================
static thread_local std::string g_last_error = "";

static int set_err(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

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
    float scale;            // mvScaleFactor[l]
    float size;             // (int)(31 * mvScaleFactor[l])
};

struct Geom {
    int L;
    int nCells;        // cells per frame (all levels)
    int candPerFrame;  // candidate slots per frame (u32)
    int kpCap;         // keypoint slots per frame (sum of nDesired)
    int fastTh, tmin;  // clamped fastTh, min(fastTh, 7)
    int scoreType;
    int taps[4];       // Gaussian 7-tap fixed-point kernel, centre first: 55, 49, 34, 18
    int umax[16];
    LevelGeom lv[ORB_MAX_LEVELS];
};

struct CellGeom {
    int level;
    int x0, y0, hx, hy;  // ROI in level coordinates (reference iniX, iniY, hX, hY)
    int cap;             // max NMS survivors: ceil(dw/2) * ceil(dh/2)
    int candOff;         // offset in the frame's candidate area
    int skipped;         // reference `continue` on hX/hY <= 0 (nTotal stays 0, bNoMore false)
};

// ======================================================================================
// kernels
// ======================================================================================
using namespace orbdev;

__constant__ signed char c_pattern[1024];

// ---- pyramid --------------------------------------------------------------------------
// Level 0: copyMakeBorder(image, 16, BORDER_REFLECT_101); one thread per 4 output bytes.
__global__ void __launch_bounds__(256) k_pyr0(const uint8_t* __restrict__ imgs, int stride, long long fpitch,
                                              uint8_t* __restrict__ pyr, Geom g) {
    const LevelGeom& lg = g.lv[0];
    const int b = blockIdx.z, py = blockIdx.y;
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (x4 >= lg.pitch) return;
    const uint8_t* src = imgs + (long long)b * fpitch + (long long)reflect101(py - EDGE, lg.h) * stride;
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int px = x4 + i;
        uint32_t v = 0;
        if (px < lg.w + 2 * EDGE) v = src[reflect101(px - EDGE, lg.w)];
        word |= v << (8 * i);
    }
    *(uint32_t*)(pyr + lg.base + (long long)b * lg.fstride + (long long)py * lg.pitch + x4) = word;
}

// Level l >= 1: cv::resize(level l-1, (w_l, h_l), INTER_LINEAR) for 8U:
// fixed-point HResizeLinear rows; vertical SSE2 body (VResizeLinearVec_32s8u) for x < xs,
// scalar FixedPtCast<int,uchar,22> tail; then copyMakeBorder(REFLECT_101 | ISOLATED), fused
// by evaluating the resize at the reflected coordinate of every padded pixel.
__global__ void __launch_bounds__(256) k_pyr_resize(uint8_t* __restrict__ pyr, const int* __restrict__ rtab, Geom g,
                                                    int l) {
    const LevelGeom& lg = g.lv[l];
    const LevelGeom& ls = g.lv[l - 1];
    const int b = blockIdx.z, py = blockIdx.y;
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (x4 >= lg.pitch) return;
    const int* xofs = rtab + lg.rtab;
    const int* alpha = xofs + lg.w;
    const int* yofs = alpha + lg.w;
    const int* beta = yofs + lg.h;
    const int ly = reflect101(py - EDGE, lg.h);
    const int sy = yofs[ly];
    const int r0 = min(max(sy, 0), ls.h - 1), r1 = min(max(sy + 1, 0), ls.h - 1);
    const int bb = beta[ly];
    const int b0 = (short)(bb & 0xFFFF), b1 = (short)(bb >> 16);
    const uint8_t* S = pyr + ls.base + (long long)b * ls.fstride + (long long)EDGE * ls.pitch + EDGE;
    const uint8_t* S0 = S + (long long)r0 * ls.pitch;
    const uint8_t* S1 = S + (long long)r1 * ls.pitch;
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int px = x4 + i;
        uint32_t v = 0;
        if (px < lg.w + 2 * EDGE) {
            int lx = reflect101(px - EDGE, lg.w);
            int sx = xofs[lx];
            int H0, H1;
            if (lx < lg.xmax) {
                int aa = alpha[lx];
                int a0 = (short)(aa & 0xFFFF), a1 = (short)(aa >> 16);
                H0 = S0[sx] * a0 + S0[sx + 1] * a1;
                H1 = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                H0 = S0[sx] * 2048;
                H1 = S1[sx] * 2048;
            }
            int r;
            if (lx < lg.xs_resize) {
                int h0 = min(max(H0 >> 4, -32768), 32767), h1 = min(max(H1 >> 4, -32768), 32767);
                int s = min(max(((h0 * b0) >> 16) + ((h1 * b1) >> 16), -32768), 32767);
                s = min(max(s + 2, -32768), 32767);
                r = s >> 2;
            } else {
                r = (H0 * b0 + H1 * b1 + (1 << 21)) >> 22;
            }
            v = (uint32_t)min(max(r, 0), 255);
        }
        word |= v << (8 * i);
    }
    *(uint32_t*)(pyr + lg.base + (long long)b * lg.fstride + (long long)py * lg.pitch + x4) = word;
}

// ---- FAST per cell ----------------------------------------------------------------------
// One workgroup per (cell, frame).  The cell ROI (cell + 3 px on each side) is staged in
// LDS; S(p) is computed for the detection region [3, hx-3) x [3, hy-3); non-max suppression
// is evaluated with out-of-region neighbours = 0, exactly as cv::FAST sees a cell-sized Mat.
// If the cell yields <= 3 corners at fastTh it is re-run at threshold 7 (ORBextractor.cc:609-614).
// Survivors are written in raster order as (score << 24) | (y << 12) | x, level coordinates.
__device__ __forceinline__ int nms_keep(const uint8_t* Sb, int dw, int dh, int xx, int yy, int t) {
    int s = Sb[yy * dw + xx];
    if (s <= t) return 0;
    int sc = s - 1;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            if (dx == 0 && dy == 0) continue;
            int nx = xx + dx, ny = yy + dy;
            int ns = 0;
            if (nx >= 0 && nx < dw && ny >= 0 && ny < dh) {
                int v = Sb[ny * dw + nx];
                ns = v > t ? v - 1 : 0;
            }
            if (!(sc > ns)) return 0;
        }
    return 1;
}

__global__ void __launch_bounds__(256) k_fast_cells(const uint8_t* __restrict__ pyr, Geom g,
                                                    const CellGeom* __restrict__ cells, uint32_t* __restrict__ cand,
                                                    int* __restrict__ cellCount) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_cnt[256];
    __shared__ int s_total;
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const CellGeom cg = cells[c];
    int* outCount = cellCount + (long long)b * g.nCells + c;
    const int dw = cg.hx - 6, dh = cg.hy - 6;
    if (cg.skipped || dw <= 0 || dh <= 0) {
        if (tid == 0) *outCount = 0;
        return;
    }
    const LevelGeom& lg = g.lv[cg.level];
    const uint8_t* roi =
        pyr + lg.base + (long long)b * lg.fstride + (long long)(EDGE + cg.y0) * lg.pitch + EDGE + cg.x0;
    const int tp = (cg.hx + 3) & ~3;
    uint8_t* tile = smem;
    uint8_t* Sb = smem + tp * cg.hy;
    for (int i = tid; i < cg.hx * cg.hy; i += 256) {
        int yy = i / cg.hx, xx = i - yy * cg.hx;
        tile[yy * tp + xx] = roi[(long long)yy * lg.pitch + xx];
    }
    __syncthreads();
    const int npix = dw * dh;
    for (int i = tid; i < npix; i += 256) {
        int yy = i / dw, xx = i - yy * dw;
        const uint8_t* p = tile + (yy + 3) * tp + (xx + 3);
        int circ[16];
        circ[0] = p[3 * tp];
        circ[1] = p[3 * tp + 1];
        circ[2] = p[2 * tp + 2];
        circ[3] = p[tp + 3];
        circ[4] = p[3];
        circ[5] = p[-tp + 3];
        circ[6] = p[-2 * tp + 2];
        circ[7] = p[-3 * tp + 1];
        circ[8] = p[-3 * tp];
        circ[9] = p[-3 * tp - 1];
        circ[10] = p[-2 * tp - 2];
        circ[11] = p[-tp - 3];
        circ[12] = p[-3];
        circ[13] = p[tp - 3];
        circ[14] = p[2 * tp - 2];
        circ[15] = p[3 * tp - 1];
        Sb[i] = (uint8_t)fast_strength(p[0], circ, g.tmin);
    }
    __syncthreads();
    // raster-order chunk per thread for the ordered compaction
    const int chunk = (npix + 255) / 256;
    const int p0 = min(tid * chunk, npix), p1 = min(p0 + chunk, npix);
    int t = g.fastTh;
    int mine = 0;
    for (int i = p0; i < p1; ++i) {
        int yy = i / dw, xx = i - yy * dw;
        mine += nms_keep(Sb, dw, dh, xx, yy, t);
    }
    s_cnt[tid] = mine;
    __syncthreads();
    if (tid == 0) {
        int s = 0;
        for (int i = 0; i < 256; ++i) s += s_cnt[i];
        s_total = s;
    }
    __syncthreads();
    if (s_total <= 3) {
        t = 7;
        mine = 0;
        for (int i = p0; i < p1; ++i) {
            int yy = i / dw, xx = i - yy * dw;
            mine += nms_keep(Sb, dw, dh, xx, yy, t);
        }
        __syncthreads();
        s_cnt[tid] = mine;
        __syncthreads();
        if (tid == 0) {
            int s = 0;
            for (int i = 0; i < 256; ++i) s += s_cnt[i];
            s_total = s;
        }
        __syncthreads();
    }
    // exclusive scan of per-thread counts (256 entries, one wave does it)
    if (tid < 64) {
        int v0 = s_cnt[4 * tid], v1 = s_cnt[4 * tid + 1], v2 = s_cnt[4 * tid + 2], v3 = s_cnt[4 * tid + 3];
        int sum = v0 + v1 + v2 + v3, incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int n = __shfl_up(incl, o, 64);
            if (tid >= o) incl += n;
        }
        int ex = incl - sum;
        s_cnt[4 * tid] = ex;
        s_cnt[4 * tid + 1] = ex + v0;
        s_cnt[4 * tid + 2] = ex + v0 + v1;
        s_cnt[4 * tid + 3] = ex + v0 + v1 + v2;
    }
    __syncthreads();
    uint32_t* out = cand + (long long)b * g.candPerFrame + cg.candOff;
    int pos = s_cnt[tid];
    for (int i = p0; i < p1; ++i) {
        int yy = i / dw, xx = i - yy * dw;
        if (nms_keep(Sb, dw, dh, xx, yy, t)) {
            int sc = Sb[i] - 1;
            int lx = cg.x0 + 3 + xx, ly = cg.y0 + 3 + yy;
            out[pos++] = ((uint32_t)sc << 24) | ((uint32_t)ly << 12) | (uint32_t)lx;
        }
    }
    if (tid == 0) *outCount = s_total;
}

// ---- selection (retainBest replay) -------------------------------------------------------
struct ScoreGreater {  // KeypointResponseGreater on the packed FAST score
    ORB_HD bool operator()(uint32_t a, uint32_t b) const { return (a >> 24) > (b >> 24); }
};

// One wave per (level, frame).
__global__ void __launch_bounds__(64) k_select(uint32_t* __restrict__ cand, const int* __restrict__ cellCount, Geom g,
                                               const CellGeom* __restrict__ cells, uint32_t* __restrict__ lvlOut,
                                               int* __restrict__ lvlCount) {
    __shared__ int s_cnt[ORB_MAX_CELLS_PER_LEVEL];
    __shared__ int s_ret[ORB_MAX_CELLS_PER_LEVEL];
    __shared__ int s_off[ORB_MAX_CELLS_PER_LEVEL + 1];
    __shared__ uint32_t s_list[ORB_SELECT_LDS_CAP];
    const int l = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const LevelGeom& lg = g.lv[l];
    const int nC = lg.rows * lg.cols;
    const CellGeom* lc = cells + lg.cell0;
    uint32_t* fcand = cand + (long long)b * g.candPerFrame;
    for (int c = lane; c < nC; c += 64) s_cnt[c] = cellCount[(long long)b * g.nCells + lg.cell0 + c];
    __syncthreads();
    if (lane == 0) {
        // nToRetain / nToDistribute / bNoMore bookkeeping (ORBextractor.cc:622-670)
        const int nfc = lg.nfc;
        int nNoMore = 0, nToDistribute = 0;
        unsigned long long noMore[(ORB_MAX_CELLS_PER_LEVEL + 63) / 64] = {};
        for (int c = 0; c < nC; ++c) {
            if (lc[c].skipped) {
                s_ret[c] = 0;
                continue;
            }
            int nKeys = s_cnt[c];
            if (nKeys > nfc) {
                s_ret[c] = nfc;
            } else {
                s_ret[c] = nKeys;
                nToDistribute += nfc - nKeys;
                noMore[c >> 6] |= 1ull << (c & 63);
                nNoMore++;
            }
        }
        while (nToDistribute > 0 && nNoMore < nC) {
            int nNew = nfc + (int)ceilf((float)nToDistribute / (nC - nNoMore));
            nToDistribute = 0;
            for (int c = 0; c < nC; ++c) {
                if (noMore[c >> 6] & (1ull << (c & 63))) continue;
                int tot = lc[c].skipped ? 0 : s_cnt[c];
                if (tot > nNew) {
                    s_ret[c] = nNew;
                } else {
                    s_ret[c] = tot;
                    nToDistribute += nNew - tot;
                    noMore[c >> 6] |= 1ull << (c & 63);
                    nNoMore++;
                }
            }
        }
    }
    __syncthreads();
    ScoreGreater comp;
    for (int c = lane; c < nC; c += 64) {
        int n = lc[c].skipped ? 0 : s_cnt[c];
        s_cnt[c] = orbsel::retain_best(fcand + lc[c].candOff, n, s_ret[c], comp);
    }
    __syncthreads();
    if (lane == 0) {
        int s = 0;
        for (int c = 0; c < nC; ++c) {
            s_off[c] = s;
            s += s_cnt[c];
        }
        s_off[nC] = s;
    }
    __syncthreads();
    const int M = s_off[nC];
    uint32_t* list;
    if (M <= ORB_SELECT_LDS_CAP) {
        for (int c = 0; c < nC; ++c) {
            const uint32_t* src = fcand + lc[c].candOff;
            for (int k = lane; k < s_cnt[c]; k += 64) s_list[s_off[c] + k] = src[k];
        }
        list = s_list;
    } else {  // sequential in-place compaction (dest <= src, ascending) into the level's area
        list = fcand + lc[0].candOff;
        if (lane == 0)
            for (int c = 0; c < nC; ++c) {
                const uint32_t* src = fcand + lc[c].candOff;
                for (int k = 0; k < s_cnt[c]; ++k) list[s_off[c] + k] = src[k];
            }
    }
    __syncthreads();
    int keep = M;
    if (M > lg.nDesired) {
        keep = lg.nDesired;
        if (lane == 0) orbsel::retain_best(list, M, lg.nDesired, comp);
    }
    __syncthreads();
    uint32_t* out = lvlOut + (long long)b * g.kpCap + lg.kpBase;
    for (int k = lane; k < keep; k += 64) out[k] = list[k];
    if (lane == 0) lvlCount[(long long)b * g.L + l] = keep;
}

// ---- orientation + descriptor -------------------------------------------------------------
// One wave per keypoint.  A 43x43 patch around the keypoint (the 31x31 IC disc, the rBRIEF
// samples' |offset| <= 18 and the 7x7 blur taps) is staged in LDS from the padded level.
#define DESC_R 21
#define DESC_P 43
#define DESC_PITCH 44

__global__ void __launch_bounds__(256) k_orient_desc(const uint8_t* __restrict__ pyr, Geom g,
                                                     const uint32_t* __restrict__ lvlOut,
                                                     const int* __restrict__ lvlCount, orb_keypoint_t* __restrict__ kps,
                                                     uint8_t* __restrict__ desc, int* __restrict__ counts) {
    __shared__ __attribute__((aligned(16))) uint8_t s_patch[4][DESC_P * DESC_PITCH];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    const int k = blockIdx.x * 4 + wave;
    // locate the level of keypoint k (level-major output order, ORBextractor.cc:749-778)
    int l = -1, off = 0, total = 0, idx = 0;
    for (int i = 0; i < g.L; ++i) {
        int cnt = lvlCount[(long long)b * g.L + i];
        if (l < 0 && k < total + cnt) {
            l = i;
            idx = k - total;
            off = total;
        }
        total += cnt;
    }
    if (k == 0 && lane == 0) counts[b] = total;
    (void)off;
    const bool valid = l >= 0;  // wave-uniform; every wave still reaches the barrier below
    const LevelGeom& lg = g.lv[valid ? l : 0];
    const uint32_t e = valid ? lvlOut[(long long)b * g.kpCap + lg.kpBase + idx] : 0u;
    const int x = e & 0xFFF, y = (e >> 12) & 0xFFF, score = e >> 24;
    const uint8_t* lvl = pyr + lg.base + (long long)b * lg.fstride;
    uint8_t* P = s_patch[wave];
    // patch rows y-21 .. y+21, cols x-21 .. x+21 (padded coordinates +16)
    if (valid)
        for (int i = lane; i < DESC_P * DESC_P; i += 64) {
            int r = i / DESC_P, cc = i - r * DESC_P;
            P[r * DESC_PITCH + cc] = lvl[(long long)(y + EDGE - DESC_R + r) * lg.pitch + (x + EDGE - DESC_R + cc)];
        }
    __syncthreads();
    if (!valid) return;
    // IC_Angle (ORBextractor.cc:124-151): lanes 0..30 take rows v = lane - 15
    int m01 = 0, m10 = 0;
    if (lane < 31) {
        int v = lane - HALF_PATCH;
        int d = g.umax[v < 0 ? -v : v];
        const uint8_t* row = P + (DESC_R + v) * DESC_PITCH + DESC_R;
        int su = 0, s = 0;
        for (int u = -d; u <= d; ++u) {
            int val = row[u];
            su += u * val;
            s += val;
        }
        m10 = su;
        m01 = v * s;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        m01 += __shfl_xor(m01, o, 64);
        m10 += __shfl_xor(m10, o, 64);
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    // computeOrbDescriptor (ORBextractor.cc:155-194)
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float sa, ca;
    glibc_sincosf(angle * factorPI, &sa, &ca);
    const float a = ca, bsin = sa;
    const int k0 = g.taps[0], k1 = g.taps[1], k2 = g.taps[2], k3 = g.taps[3];
    auto sample = [&](int idx_pt) -> int {
        float px = (float)c_pattern[2 * idx_pt], py = (float)c_pattern[2 * idx_pt + 1];
        int dy = (int)rintf(__builtin_fmaf(px, bsin, py * a));
        int dx = (int)rintf(__builtin_fmaf(px, a, -(py * bsin)));
        int sx = x + dx, sy = y + dy;
        const uint8_t* q = P + (DESC_R + dy) * DESC_PITCH + (DESC_R + dx);
        if (sx < 0 || sx >= lg.w || sy < 0 || sy >= lg.h) return q[0];  // un-blurred padding
        int T = 0;
#pragma unroll
        for (int j = -3; j <= 3; ++j) {
            const uint8_t* r = q + j * DESC_PITCH;
            int R = k0 * r[0] + k1 * (r[-1] + r[1]) + k2 * (r[-2] + r[2]) + k3 * (r[-3] + r[3]);
            int kj = j == 0 ? k0 : (j == 1 || j == -1) ? k1 : (j == 2 || j == -2) ? k2 : k3;
            T += kj * R;
        }
        int v = sx < lg.xsimd_blur ? (T + 32767 + ((T >> 16) & 1)) >> 16 : (T + 32768) >> 16;
        return min(v, 255);
    };
    int nib = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int test = lane * 4 + q;  // bit (test & 7) of byte test >> 3
        int t0 = sample(2 * test), t1 = sample(2 * test + 1);
        nib |= (t0 < t1) << q;
    }
    int other = __shfl_xor(nib, 1, 64);
    const long long kslot = (long long)b * g.kpCap + k;
    if ((lane & 1) == 0) desc[kslot * 32 + (lane >> 1)] = (uint8_t)(nib | (other << 4));
    if (lane == 0) {
        orb_keypoint_t kp;
        kp.x = l == 0 ? (float)x : (float)x * lg.scale;
        kp.y = l == 0 ? (float)y : (float)y * lg.scale;
        kp.size = lg.size;
        kp.angle = angle;
        kp.response = (float)score;
        kp.octave = l;
        kp.class_id = -1;
        kps[kslot] = kp;
    }
}

// ---- SearchForInitialization ------------------------------------------------------------
struct MatchGeom {
    int minX, maxX, minY, maxY;
    float invW, invH;  // FRAME_GRID_COLS / (maxX - minX), FRAME_GRID_ROWS / (maxY - minY)
};

// One wave per frame pair.  F2's octave-0, in-grid keypoints (the only possible candidates of
// GetFeaturesInArea(x, y, window, 0, 0), Frame.cc:200-265) are staged in LDS with their grid
// cell; F1's octave-0 keypoints are then processed in index order, sequentially, as the
// reference's greedy loop requires (vMatchedDistance / vnMatches21 feed later queries).  For
// each query the candidate set is evaluated in parallel and reduced to (best, first-in-grid-
// traversal-order argmin, second-best) — the values the reference's sequential scan produces.
__global__ void __launch_bounds__(64) k_match_init(const orb_keypoint_t* __restrict__ kps,
                                                   const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                   int cap, int n2max, const int* __restrict__ pf1,
                                                   const int* __restrict__ pf2, MatchGeom mg, float nnratio,
                                                   int checkOri, float r, float* __restrict__ prev,
                                                   int* __restrict__ m12out, int* __restrict__ nmOut) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int p = blockIdx.x, lane = threadIdx.x;
    const int f1 = pf1[p], f2 = pf2[p];
    const int n1 = counts[f1], n2 = counts[f2];
    const orb_keypoint_t* K1 = kps + (long long)f1 * cap;
    const orb_keypoint_t* K2 = kps + (long long)f2 * cap;
    const uint32_t* D1 = (const uint32_t*)(desc + (long long)f1 * cap * 32);
    const uint32_t* D2 = (const uint32_t*)(desc + (long long)f2 * cap * 32);
    uint32_t* s_d2 = (uint32_t*)smem;                    // n2max x 8
    float* s_x2 = (float*)(s_d2 + (size_t)n2max * 8);    // n2max
    float* s_y2 = s_x2 + n2max;                          // n2max
    int* s_cell = (int*)(s_y2 + n2max);                  // posX * 48 + posY
    int* s_idx = s_cell + n2max;                         // original index i2
    int* s_md = s_idx + n2max;                           // vMatchedDistance
    int* s_m21 = s_md + n2max;                           // vnMatches21
    int* s_m12 = s_m21 + n2max;                          // vnMatches12 (cap)
    signed char* s_bin = (signed char*)(s_m12 + cap);    // rotation bin of accepted i1 (cap)
    __shared__ int s_n2c;
    __shared__ int s_hist[32];
    __shared__ int s_ind[3];
    // stage F2 candidates (octave 0, PosInGrid true), preserving index order
    int base = 0;
    for (int i0 = 0; i0 < n2; i0 += 64) {
        int i2 = i0 + lane;
        bool ok = false;
        int px = 0, py = 0;
        if (i2 < n2) {
            orb_keypoint_t kp = K2[i2];
            px = (int)roundf((kp.x - mg.minX) * mg.invW);
            py = (int)roundf((kp.y - mg.minY) * mg.invH);
            ok = kp.octave == 0 && !(px < 0 || px >= 64 || py < 0 || py >= 48);
        }
        unsigned long long m = __ballot(ok);
        int slot = base + __popcll(m & ((1ull << lane) - 1ull));
        if (ok && slot < n2max) {
            orb_keypoint_t kp = K2[i2];
            s_x2[slot] = kp.x;
            s_y2[slot] = kp.y;
            s_cell[slot] = px * 48 + py;
            s_idx[slot] = i2;
            s_md[slot] = 0x7fffffff;
            s_m21[slot] = -1;
#pragma unroll
            for (int w = 0; w < 8; ++w) s_d2[slot * 8 + w] = D2[(long long)i2 * 8 + w];
        }
        base += __popcll(m);
    }
    if (lane == 0) s_n2c = min(base, n2max);
    for (int i = lane; i < n1; i += 64) {
        s_m12[i] = -1;
        s_bin[i] = -1;
    }
    __syncthreads();
    const int n2c = s_n2c;
    for (int i1 = 0; i1 < n1; ++i1) {
        const orb_keypoint_t kp1 = K1[i1];
        if (kp1.octave != 0) continue;  // level1 > 0 (octave < 0 rejected by the host API)
        const float qx = prev ? prev[((long long)p * cap + i1) * 2] : kp1.x;
        const float qy = prev ? prev[((long long)p * cap + i1) * 2 + 1] : kp1.y;
        int minCX = max(0, (int)floorf((qx - mg.minX - r) * mg.invW));
        int maxCX = min(63, (int)ceilf((qx - mg.minX + r) * mg.invW));
        int minCY = max(0, (int)floorf((qy - mg.minY - r) * mg.invH));
        int maxCY = min(47, (int)ceilf((qy - mg.minY + r) * mg.invH));
        if (minCX > maxCX || minCY > maxCY) continue;
        uint32_t d1[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) d1[w] = D1[(long long)i1 * 8 + w];
        // lane-local best (dist, traversal order, slot) and second-best distance
        unsigned long long lbest = ~0ull;
        int lsecond = 0x7fffffff;
        for (int j = lane; j < n2c; j += 64) {
            int cell = s_cell[j];
            int cx = cell / 48, cy = cell - cx * 48;
            if (cx < minCX || cx > maxCX || cy < minCY || cy > maxCY) continue;
            if (fabsf(s_x2[j] - qx) > r || fabsf(s_y2[j] - qy) > r) continue;
            int dist = hamming256(d1, s_d2 + j * 8);
            if (s_md[j] <= dist) continue;
            unsigned long long key = ((unsigned long long)dist << 40) |
                                     ((unsigned long long)((cell << 16) | s_idx[j]) << 11) | (unsigned long long)j;
            if (key < lbest) {
                if (lbest != ~0ull) lsecond = (int)(lbest >> 40);
                lbest = key;
            } else if (dist < lsecond) {
                lsecond = dist;
            }
        }
        unsigned long long gbest = lbest;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            unsigned long long v = __shfl_xor(gbest, o, 64);
            gbest = v < gbest ? v : gbest;
        }
        if (gbest == ~0ull) continue;  // no candidate
        int contrib = (lbest == gbest) ? lsecond : (lbest == ~0ull ? 0x7fffffff : (int)(lbest >> 40));
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) contrib = min(contrib, __shfl_xor(contrib, o, 64));
        const int bestDist = (int)(gbest >> 40);
        const int bestSlot = (int)(gbest & 0x7FF);
        if (bestDist <= 50 && (float)bestDist < (float)contrib * nnratio) {
            if (lane == 0) {
                const int bestIdx2 = s_idx[bestSlot];
                int old = s_m21[bestSlot];
                if (old >= 0) s_m12[old] = -1;
                s_m12[i1] = bestIdx2;
                s_m21[bestSlot] = i1;
                s_md[bestSlot] = bestDist;
                if (checkOri) {
                    float rot = kp1.angle - K2[bestIdx2].angle;
                    if (rot < 0.0f) rot += 360.0f;
                    int bin = (int)roundf(rot * (1.0f / 30));
                    if (bin == 30) bin = 0;
                    s_bin[i1] = (signed char)bin;
                }
            }
            __syncthreads();
        }
    }
    __syncthreads();
    if (checkOri) {
        if (lane < 32) s_hist[lane] = 0;
        __syncthreads();
        for (int i = lane; i < n1; i += 64)
            if (s_bin[i] >= 0) atomicAdd(&s_hist[(int)s_bin[i]], 1);
        __syncthreads();
        if (lane == 0) {  // ComputeThreeMaxima (ORBmatcher.cc:1748-1789)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < 30; ++i) {
                const int s = s_hist[i];
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
            s_ind[0] = ind1;
            s_ind[1] = ind2;
            s_ind[2] = ind3;
        }
        __syncthreads();
        const int i1x = s_ind[0], i2x = s_ind[1], i3x = s_ind[2];
        for (int i = lane; i < n1; i += 64) {
            int bn = s_bin[i];
            if (bn >= 0 && bn != i1x && bn != i2x && bn != i3x) s_m12[i] = -1;
        }
        __syncthreads();
    }
    int nm = 0;
    for (int i = lane; i < n1; i += 64) {
        int m = s_m12[i];
        m12out[(long long)p * cap + i] = m;
        if (m >= 0) {
            nm++;
            if (prev) {
                prev[((long long)p * cap + i) * 2] = K2[m].x;
                prev[((long long)p * cap + i) * 2 + 1] = K2[m].y;
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) nm += __shfl_xor(nm, o, 64);
    if (lane == 0) nmOut[p] = nm;
}

// ======================================================================================
// host side
// ======================================================================================
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
    hipStream_t stream = nullptr;
    // geometry of the current frame size
    int W = 0, H = 0;
    Geom g{};
    std::vector<CellGeom> cells;
    std::vector<int> rtab;
    size_t cellLds = 0;
    // device workspace
    uint8_t* d_pyr = nullptr;
    uint32_t* d_cand = nullptr;
    int* d_cellCount = nullptr;
    uint32_t* d_lvl = nullptr;
    int* d_lvlCount = nullptr;
    int* d_rtab = nullptr;
    CellGeom* d_cells = nullptr;
    // per-stage HIP-event timing (orb_profile_*): stage k brackets its kernel(s) on the launch stream
    static constexpr int kStages = 5;
    bool prof = false;
    std::vector<hipEvent_t> evPool;  // 2 per stage per launch, recycled after each read
    std::vector<std::pair<int, int>> evPending;  // (stage, index of the start event)
    double stageMs[kStages] = {};
    long long stageLaunches[kStages] = {};
    int evNext = 0;
    // staging for host-buffer entry points
    uint8_t* d_img = nullptr;
    orb_keypoint_t* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_counts = nullptr;

    void free_events() {
        for (auto e : evPool) hipEventDestroy(e);
        evPool.clear();
        evPending.clear();
        evNext = 0;
    }

    void free_ws() {
        hipFree(d_pyr);
        hipFree(d_cand);
        hipFree(d_cellCount);
        hipFree(d_lvl);
        hipFree(d_lvlCount);
        hipFree(d_rtab);
        hipFree(d_cells);
        hipFree(d_img);
        hipFree(d_kps);
        hipFree(d_desc);
        hipFree(d_counts);
        d_pyr = nullptr;
        d_cand = nullptr;
        d_cellCount = nullptr;
        d_lvl = nullptr;
        d_lvlCount = nullptr;
        d_rtab = nullptr;
        d_cells = nullptr;
        d_img = nullptr;
        d_kps = nullptr;
        d_desc = nullptr;
        d_counts = nullptr;
        W = H = 0;
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
        G.tmin = std::min(G.fastTh, 7);
        G.scoreType = scoreType;
        int k7[7];
        gaussian_taps7(k7);
        for (int i = 0; i < 4; ++i) G.taps[i] = k7[3 + i];
        for (int v = 0; v < 16; ++v) G.umax[v] = umax[v];
        std::vector<CellGeom> cl;
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
                            size_t lds = (size_t)((c.hx + 3) & ~3) * c.hy + (size_t)std::max(dw, 0) * std::max(dh, 0);
                            cellLds = std::max(cellLds, lds);
                        }
                    }
                    c.candOff = cand;
                    cand += c.cap;
                    cl.push_back(c);
                }
            }
        }
        if (cellLds > 150 * 1024) return set_err(ORB_ENOTSUP, "FAST cell larger than the LDS budget");
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
            int xs = 0;
            while (xs <= dw - 16) xs += 16;
            while (xs < dw - 4) xs += 4;
            lg.xs_resize = xs;
            lg.xmax = xmax;
            rt.insert(rt.end(), xofs.begin(), xofs.end());
            rt.insert(rt.end(), alpha.begin(), alpha.end());
            rt.insert(rt.end(), yofs.begin(), yofs.end());
            rt.insert(rt.end(), beta.begin(), beta.end());
        }
        G.nCells = (int)cl.size();
        G.candPerFrame = cand;
        G.kpCap = kpCap;
        // workspace
        HIP_TRY(hipMalloc(&d_pyr, (size_t)pyrBytes));
        HIP_TRY(hipMalloc(&d_cand, (size_t)std::max(cand, 1) * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_cellCount, (size_t)G.nCells * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_lvl, (size_t)std::max(kpCap, 1) * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_lvlCount, (size_t)nlevels * maxBatch * 4));
        HIP_TRY(hipMalloc(&d_rtab, std::max<size_t>(rt.size(), 1) * 4));
        HIP_TRY(hipMalloc(&d_cells, cl.size() * sizeof(CellGeom)));
        if (!rt.empty()) HIP_TRY(hipMemcpy(d_rtab, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_cells, cl.data(), cl.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
        g = G;
        cells = std::move(cl);
        rtab = std::move(rt);
        W = w0;
        H = h0;
        return ORB_OK;
    }

    int ensure_staging() {
        if (d_img) return ORB_OK;
        HIP_TRY(hipMalloc(&d_img, (size_t)W * H * maxBatch));
        HIP_TRY(hipMalloc(&d_kps, (size_t)std::max(kpCap, 1) * maxBatch * sizeof(orb_keypoint_t)));
        HIP_TRY(hipMalloc(&d_desc, (size_t)std::max(kpCap, 1) * maxBatch * 32));
        HIP_TRY(hipMalloc(&d_counts, (size_t)maxBatch * 4));
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
    void stage_begin(int stage, hipStream_t st) {
        if (!prof) return;
        int i = evNext;
        hipEvent_t a = next_event(), b = next_event();
        if (!a || !b) return;
        hipEventRecord(a, st);
        evPending.push_back({stage, i});
    }
    void stage_end(hipStream_t st) {
        if (!prof || evPending.empty()) return;
        hipEventRecord(evPool[evPending.back().second + 1], st);
    }
    int profile_collect() {
        for (auto& pe : evPending) {
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

    int launch(int B, const uint8_t* d_imgs, int stride, long long fpitch, orb_keypoint_t* kps, uint8_t* desc,
               int* counts, hipStream_t st) {
        if (prof && evNext > 4096) {  // bound the pool between reads
            int r = profile_collect();
            if (r) return r;
        }
        stage_begin(0, st);
        {
            const LevelGeom& lg = g.lv[0];
            dim3 grid((lg.pitch / 4 + 255) / 256, lg.ph, B);
            hipLaunchKernelGGL(k_pyr0, grid, dim3(256), 0, st, d_imgs, stride, fpitch, d_pyr, g);
        }
        stage_end(st);
        stage_begin(1, st);
        for (int l = 1; l < nlevels; ++l) {
            const LevelGeom& lg = g.lv[l];
            dim3 grid((lg.pitch / 4 + 255) / 256, lg.ph, B);
            hipLaunchKernelGGL(k_pyr_resize, grid, dim3(256), 0, st, d_pyr, d_rtab, g, l);
        }
        stage_end(st);
        stage_begin(2, st);
        hipLaunchKernelGGL(k_fast_cells, dim3(g.nCells, B), dim3(256), cellLds, st, d_pyr, g, d_cells, d_cand,
                           d_cellCount);
        stage_end(st);
        stage_begin(3, st);
        hipLaunchKernelGGL(k_select, dim3(nlevels, B), dim3(64), 0, st, d_cand, d_cellCount, g, d_cells, d_lvl,
                           d_lvlCount);
        stage_end(st);
        stage_begin(4, st);
        dim3 gd((std::max(kpCap, 1) + 3) / 4, B);
        hipLaunchKernelGGL(k_orient_desc, gd, dim3(256), 0, st, d_pyr, g, d_lvl, d_lvlCount, kps, desc, counts);
        stage_end(st);
        HIP_TRY(hipGetLastError());
        return ORB_OK;
    }
};

static int upload_pattern(int device) {
    static bool uploaded[64] = {};
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (device >= 0 && device < 64 && uploaded[device]) return ORB_OK;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), kOrbPattern31, sizeof(kOrbPattern31)));
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
    if (score_type == ORB_HARRIS_SCORE) return set_err(ORB_ENOTSUP, "HARRIS_SCORE is not implemented on the GPU path yet");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(ORB_EINVAL, "device ordinal out of range");
    HIP_TRY(hipSetDevice(device));
    int st = upload_pattern(device);
    if (st) return st;
    orb_extractor* h = new orb_extractor();
    h->nfeatures = nfeatures;
    h->scaleFactor = scale_factor;
    h->nlevels = nlevels;
    h->scoreType = score_type;
    h->fastTh = fast_th;
    h->device = device;
    h->maxBatch = max_batch;
    h->init_params();
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return set_err(ORB_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = h;
    return ORB_OK;
}

int orb_extractor_destroy(orb_extractor_t* h) {
    if (!h) return ORB_OK;
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    h->free_ws();
    h->free_events();
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
    if (w != h->W || hgt != h->H) {
        HIP_TRY(hipStreamSynchronize(h->stream));
        int st = h->build_geometry(w, hgt);
        if (st) return st;
    }
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    return h->launch(B, d_imgs, stride, frame_pitch, d_kps, d_desc, d_counts, st);
}

int orb_extract_batch(orb_extractor_t* h, int B, const uint8_t* imgs, int w, int hgt, int stride, int64_t frame_pitch,
                      orb_keypoint_t* kps_out, uint8_t* desc_out, int32_t* n_out) {
    if (!h || B <= 0 || !imgs || !kps_out || !desc_out || !n_out) return set_err(ORB_EINVAL, "bad arguments");
    if (B > h->maxBatch) return set_err(ORB_EINVAL, "B exceeds max_batch");
    if (w <= 0 || hgt <= 0 || stride < w || frame_pitch < (int64_t)stride * hgt)
        return set_err(ORB_EINVAL, "bad image geometry");
    HIP_TRY(hipSetDevice(h->device));
    if (w != h->W || hgt != h->H) {
        HIP_TRY(hipStreamSynchronize(h->stream));
        int st = h->build_geometry(w, hgt);
        if (st) return st;
    }
    int st = h->ensure_staging();
    if (st) return st;
    HIP_TRY(hipMemcpy2DAsync(h->d_img, w, imgs, stride, w, (size_t)hgt, hipMemcpyHostToDevice, h->stream));
    for (int k = 1; k < B; ++k)
        HIP_TRY(hipMemcpy2DAsync(h->d_img + (size_t)k * w * hgt, w, imgs + (size_t)k * frame_pitch, stride, w,
                                 (size_t)hgt, hipMemcpyHostToDevice, h->stream));
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
    std::vector<orb_keypoint_t> k(std::max(h->kpCap, 1));
    std::vector<uint8_t> d((size_t)std::max(h->kpCap, 1) * 32);
    int32_t n = 0;
    int st = orb_extract_batch(h, 1, img, w, hgt, stride, (int64_t)stride * hgt, k.data(), d.data(), &n);
    if (st) return st;
    if (n > kps_cap) return set_err(ORB_ERANGE, "kps_cap smaller than the number of keypoints");
    std::memcpy(kps_out, k.data(), (size_t)n * sizeof(orb_keypoint_t));
    std::memcpy(desc_out, d.data(), (size_t)n * 32);
    *n_out = n;
    return ORB_OK;
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

static size_t match_lds_bytes(int cap, int n2max) {
    return (size_t)n2max * (32 + 4 * 6) + (size_t)cap * 4 + (size_t)cap + 16;
}

int orb_search_for_initialization_batch_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                               const int32_t* d_counts, int cap, int P, const int32_t* d_pair_f1,
                                               const int32_t* d_pair_f2, orb_frame_bounds_t bounds, float nnratio,
                                               int check_ori, int window, float* d_prev_xy, int32_t* d_matches12,
                                               int32_t* d_nmatches, void* stream) {
    if (!d_kps || !d_desc || !d_counts || cap <= 0 || P < 0 || !d_pair_f1 || !d_pair_f2 || !d_matches12 ||
        !d_nmatches)
        return set_err(ORB_EINVAL, "bad arguments");
    if (P == 0) return ORB_OK;
    if (bounds.max_x <= bounds.min_x || bounds.max_y <= bounds.min_y) return set_err(ORB_EINVAL, "bad bounds");
    const int n2max = std::min(cap, 2047);
    size_t lds = match_lds_bytes(cap, n2max);
    if (lds > 160 * 1024 - 256) return set_err(ORB_ENOTSUP, "per-frame keypoint capacity too large for LDS");
    MatchGeom mg{bounds.min_x, bounds.max_x, bounds.min_y, bounds.max_y,
                 static_cast<float>(64) / static_cast<float>(bounds.max_x - bounds.min_x),
                 static_cast<float>(48) / static_cast<float>(bounds.max_y - bounds.min_y)};
    hipLaunchKernelGGL(k_match_init, dim3(P), dim3(64), lds, (hipStream_t)stream, d_kps, d_desc, d_counts, cap, n2max,
                       d_pair_f1, d_pair_f2, mg, nnratio, check_ori, (float)window, d_prev_xy, d_matches12,
                       d_nmatches);
    HIP_TRY(hipGetLastError());
    return ORB_OK;
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
    if (n2 > 2047) return set_err(ORB_ENOTSUP, "F2 has more than 2047 keypoints");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    orb_keypoint_t* dk = nullptr;
    uint8_t* dd = nullptr;
    int *dc = nullptr, *dm = nullptr;
    float* dp = nullptr;
    auto cleanup = [&]() {
        hipFree(dk);
        hipFree(dd);
        hipFree(dc);
        hipFree(dm);
        hipFree(dp);
    };
    hipError_t e = hipSuccess;
    do {
        if ((e = hipMalloc(&dk, (size_t)2 * cap * sizeof(orb_keypoint_t))) != hipSuccess) break;
        if ((e = hipMalloc(&dd, (size_t)2 * cap * 32)) != hipSuccess) break;
        if ((e = hipMalloc(&dc, 6 * sizeof(int))) != hipSuccess) break;
        if ((e = hipMalloc(&dm, (size_t)cap * 4 + 4)) != hipSuccess) break;
        if ((e = hipMalloc(&dp, (size_t)cap * 8)) != hipSuccess) break;
        int hostc[6] = {n1, n2, 0, 1, 0, 0};
        if ((e = hipMemcpy(dk, kps1, (size_t)n1 * sizeof(orb_keypoint_t), hipMemcpyHostToDevice)) != hipSuccess) break;
        if (n2 && (e = hipMemcpy(dk + cap, kps2, (size_t)n2 * sizeof(orb_keypoint_t), hipMemcpyHostToDevice)) != hipSuccess)
            break;
        if ((e = hipMemcpy(dd, desc1, (size_t)n1 * 32, hipMemcpyHostToDevice)) != hipSuccess) break;
        if (n2 && (e = hipMemcpy(dd + (size_t)cap * 32, desc2, (size_t)n2 * 32, hipMemcpyHostToDevice)) != hipSuccess) break;
        if ((e = hipMemcpy(dc, hostc, sizeof(hostc), hipMemcpyHostToDevice)) != hipSuccess) break;
        if ((e = hipMemcpy(dp, prev_xy, (size_t)n1 * 8, hipMemcpyHostToDevice)) != hipSuccess) break;
    } while (0);
    if (e != hipSuccess) {
        cleanup();
        return set_err(ORB_EDEVICE, std::string("match staging: ") + hipGetErrorString(e));
    }
    int st = orb_search_for_initialization_batch_device(dk, dd, dc, cap, 1, dc + 2, dc + 3, bounds, nnratio, check_ori,
                                                        window, dp, dm, dm + cap, nullptr);
    if (st) {
        cleanup();
        return st;
    }
    int nm = 0;
    if ((e = hipDeviceSynchronize()) == hipSuccess && (e = hipMemcpy(matches12, dm, (size_t)n1 * 4, hipMemcpyDeviceToHost)) == hipSuccess &&
        (e = hipMemcpy(&nm, dm + cap, 4, hipMemcpyDeviceToHost)) == hipSuccess)
        e = hipMemcpy(prev_xy, dp, (size_t)n1 * 8, hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) return set_err(ORB_EDEVICE, std::string("match: ") + hipGetErrorString(e));
    *n_matches = nm;
    return ORB_OK;
}

static const char* kStageNames[] = {"k_pyr0", "k_pyr_resize", "k_fast_cells", "k_select", "k_orient_desc"};

int orb_profile_enable(orb_extractor_t* h, int enable) {
    if (!h) return set_err(ORB_EINVAL, "bad handle");
    HIP_TRY(hipSetDevice(h->device));
    int r = h->profile_collect();
    if (r) return r;
    h->prof = enable != 0;
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

// Per-cell FAST counts (after fallback) of frame `b`, level `l`, row-major cells.
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
