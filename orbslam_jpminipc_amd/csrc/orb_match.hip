// orb_match.hip — MI355X (gfx950) kernels for the ORBmatcher family beyond
// SearchForInitialization, plus the Frame / KeyFrame window queries they stand on.
//
// Every matcher of the reference (ORBmatcher.cc) is the same computation with different
// knobs: for each query (a MapPoint or a keypoint, in the reference's loop order) build a
// candidate list on a target frame — a 64 x 48 grid window (Frame::GetFeaturesInArea,
// KeyFrame::GetFeaturesInArea) or a shared vocabulary node (SearchByBoW) — take the Hamming
// best (and second best) of the candidates that are not yet taken, accept by a
// threshold / ratio rule, mark the target taken, and finally drop matches outside the three
// dominant rotation-histogram bins.  The GPU runs that as four kernels per call:
//
//   k_grid_build   one block per target frame: the grid as CSR (cellStart[3073], items[]) in
//                  cell order ix*48+iy, keypoint index order inside a cell = the reference's
//                  traversal order (ix outer, iy inner, insertion order).
//   k_query_prep   one thread per query: the per-query geometry (projection, frustum /
//                  image / distance / viewing-angle tests, predicted level, window radius).
//   k_query_scan   one wave per query: every candidate of the window, Hamming distance,
//                  the 8 smallest (distance, traversal order) keys and the candidate count.
//                  Targets taken before the call are skipped here (taken only grows).
//   k_resolve      one block per call: the loop-carried part.  Matchers whose candidate
//                  loop skips targets taken earlier IN THE SAME CALL (F.mvpMapPoints[idx],
//                  vpMatched[idx], vbMatched2[idx]) replay the queries in order on one wave:
//                  best / second = the first untaken entries of the query's top-8; if the
//                  top-8 runs out the wave rescans the full window against the live taken
//                  flags (exact).  Then the rotation histogram / ComputeThreeMaxima filter.
//                  Matchers without that dependency (Fuse, SearchBySim3) resolve in parallel.
//
// Arithmetic follows the reference bit for bit: cv::Mat algebra (gemm fast path, norm, dot)
// in the double/float mix OpenCV 2.4 uses, the reference's own float expressions with the
// FMA contraction g++ -O3 -march=native applies (explicit __builtin_fmaf; see
// scripts/contraction_check.sh), IEEE division/sqrt (-fhip-fp32-correctly-rounded-divide-sqrt).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"
#include "orb_device.h"
#include "orb_internal.h"

using orbdev::hamming256;
using orbdev::min8;

namespace {

constexpr int GRID_COLS = 64, GRID_ROWS = 48, NCELLS = GRID_COLS * GRID_ROWS;  // Frame.h:35-36
constexpr int TOPK = 8;
constexpr int TOPK_FIX = 32;  // the fixed-point resolver's lists (fewer exact rescans)
constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO = 30;  // ORBmatcher.cc:40-42
constexpr int MAX_TARGET = 16384;                       // keypoints per target frame (LDS state)
static_assert(NCELLS == 3 * 1024 && MAX_TARGET <= 65536, "k_grid_build: 3 cells per thread, u16 item indices");

enum Mode : int {
    M_AREA_F = 0,   // Frame::GetFeaturesInArea
    M_AREA_KF,      // KeyFrame::GetFeaturesInArea
    M_LOCAL,        // SearchByProjection(Frame&, vector<MapPoint*>, th)       ORBmatcher.cc:49-125
    M_WINDOW,       // WindowSearch                                            409-516
    M_F2F,          // SearchByProjection(Frame&, Frame&, windowSize, ...)     519-594
    M_MOTION,       // SearchByProjection(Frame&, const Frame&, th)            1507-1620
    M_RELOC,        // SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist) 1622-1746
    M_SIM3P,        // SearchByProjection(KeyFrame*, Scw, ...)                 286-407
    M_FUSE,         // Fuse(KeyFrame*, vector<MapPoint*>, th)                  1016-1134
    M_FUSE_SCW,     // Fuse(KeyFrame*, Scw, vpPoints, th)                      1136-1265
    M_SIM3,         // one direction of SearchBySim3                           1267-1505
    M_BOW_KFF,      // SearchByBoW(KeyFrame*, Frame&)                          155-284
    M_BOW_KFKF,     // SearchByBoW(KeyFrame*, KeyFrame*)                       715-850
    M_TRIANG,       // SearchForTriangulation                                  852-1014
};

__host__ __device__ constexpr bool is_bow(int m) { return m == M_BOW_KFF || m == M_BOW_KFKF || m == M_TRIANG; }
// candidate loop skips targets taken earlier in the same call -> sequential replay
__host__ __device__ constexpr bool is_exclusive(int m) {
    return m == M_LOCAL || m == M_WINDOW || m == M_F2F || m == M_MOTION || m == M_RELOC || m == M_SIM3P ||
           m == M_BOW_KFF || m == M_BOW_KFKF || m == M_TRIANG;
}
// best and second best (ratio test) vs best only
__host__ __device__ constexpr bool needs_second(int m) {
    return m == M_LOCAL || m == M_WINDOW || m == M_F2F || m == M_BOW_KFF || m == M_BOW_KFKF;
}

// Target frame on the device.
struct DView {
    const orb_keypoint_t* kps;
    const uint32_t* desc;  // n x 8
    int n, nlevels;
    int minX, maxX, minY, maxY;
    float invW, invH;  // mfGridElementWidthInv / HeightInv (Frame.cc:77-78)
    float sf[ORB_MAX_VIEW_LEVELS], sigma2[ORB_MAX_VIEW_LEVELS];
    float fx, fy, cx, cy;
    float R[9], t[3], Ow[3];
    const int* cellStart;  // NCELLS + 1 (grid modes)
    const int* items;      // grid: keypoint indices in traversal order; BoW: FV2 feature array
};

// Per-query window.  flags: 1 valid, 2 KeyFrame-style area (no level filter, <= r),
// 4 post level filter [pMin, pMax] (KeyFrame matchers' kpLevel test)
struct QP {
    float u, v, r;
    int flags;
    int aMin, aMax;  // Frame::GetFeaturesInArea minLevel / maxLevel
    int pMin, pMax;
    int lo, hi;      // BoW: candidate range in DView::items
};

struct Job {
    int mode;
    DView T;
    int qn;
    const uint8_t* qflag;        // per query-side element: usable (TRIANG: has MapPoint)
    const uint32_t* qdesc;       // query-side descriptor rows (x 8)
    const orb_keypoint_t* qkps;  // query-side keypoints
    const float* qpos;
    const float* qnormal;
    const float* qdmin;
    const float* qdmax;
    const float* qu;   // LOCAL: mTrackProjX; AREA: x
    const float* qv;
    const int* qlevel;  // LOCAL: mnTrackScaleLevel; AREA: (min, max) pairs
    const float* qvcos;  // LOCAL: mTrackViewCos; AREA: r
    float th, nnratio;
    int window, minLevel, maxLevel, thDist, checkOri;
    float SR[9], St[3];          // SIM3: sim transform applied after the source pose
    float SRw[9], Stw[3];        // SIM3: source keyframe pose (R1w, t1w)
    float qfx, qfy, qcx, qcy;    // SIM3: calibration of the projection (pKF1's)
    float F12[9];
    const uint8_t* tflag;        // BOW_KFKF: target usable; TRIANG: target has MapPoint
    // BoW: query q = position in FV1's feature array
    const uint32_t* fv1Nodes;
    const int* fv1Off;
    const int* fv1Feat;
    int fv1N;
    const uint32_t* fv2Nodes;
    const int* fv2Off;
    int fv2N;
    // state, scratch, outputs
    const uint8_t* taken0;  // T.n exclusion flags on entry (NULL = none)
    QP* qp;
    uint32_t* topk;  // qn x topS (allocated qn x TOPK_FIX)
    uint32_t* topx;  // qn x topS: target index | octave << 24 of each entry (k_query_scan)
    int topS;        // list length / stride: TOPK (k_resolve) or TOPK_FIX (k_resolve_fix)
    int* kval;       // (topS == TOPK_FIX) per query: the list's exact prefix (entries past it may be missing)
    int* cnt;        // qn
    int* out;        // outN
    int outN, outByTarget;
    int* nOut;       // [0] = nmatches
    int* areaOff;    // AREA fill: qn + 1 offsets
    int* areaOut;
};

__device__ __forceinline__ int qrow(const Job& J, int q) { return is_bow(J.mode) ? J.fv1Feat[q] : q; }

// ---- OpenCV 2.4 cv::Mat algebra on 3-vectors (oracle/ocv_ops.h states the semantics) ----
__device__ __forceinline__ void gemm3_add(const float* A, const float* x, const float* t, float* o) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float ti = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
        o[i] = (float)((double)ti * 1.0 + (double)t[i] * 1.0);
    }
}
__device__ __forceinline__ double norm3(const float* v) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double e = v[i];
        s += e * e;
    }
    return sqrt(s);
}
__device__ __forceinline__ double dot3(const float* a, const float* b) {
    double r = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) r += (double)a[i] * (double)b[i];
    return r;
}
__device__ __forceinline__ int predict_level(const DView& T, float ratio) {  // lower_bound, clamped
    int n = 0;
    while (n < T.nlevels && T.sf[n] < ratio) ++n;
    return min(n, T.nlevels - 1);
}
__device__ __forceinline__ bool kf_in_image(const DView& T, float x, float y) {  // KeyFrame.cc:654-657
    return x >= (float)T.minX && x < (float)T.maxX && y >= (float)T.minY && y < (float)T.maxY;
}
__device__ __forceinline__ int rot_bin(float a1, float a2) {  // ORBmatcher.cc:668-675
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / HISTO));
    if (bin == HISTO) bin = 0;
    return bin;
}
__device__ __forceinline__ void load_desc(const uint32_t* p, uint32_t (&d)[8]) {
    const uint4 a = *(const uint4*)p, b = *(const uint4*)(p + 4);
    d[0] = a.x, d[1] = a.y, d[2] = a.z, d[3] = a.w, d[4] = b.x, d[5] = b.y, d[6] = b.z, d[7] = b.w;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return orbdev::wave_min_u32(v); }
__device__ __forceinline__ int wave_sum(int v) { return orbdev::wave_total(v); }
// Insert key into the sorted list t, keeping the smallest entries: the new t[i] is the median
// of (old t[i-1], key, old t[i]) -- one v_med3_u32 per entry, all independent (the min / max
// insertion chain was two dependent ops per entry)
__device__ __forceinline__ void topk_insert(uint32_t (&t)[TOPK], uint32_t key) {
#pragma unroll
    for (int i = TOPK - 1; i >= 1; --i) {
        uint32_t r;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(t[i - 1]), "v"(key), "v"(t[i]));
        t[i] = r;
    }
    t[0] = min(t[0], key);
}

// ---- k_grid_build ------------------------------------------------------------------------
// Frame::PosInGrid (Frame.cc:267-277) for every keypoint; CSR in cell order, keypoint order
// inside a cell (the reference pushes back in index order, Frame.cc:117-123).
__global__ void __launch_bounds__(1024) k_grid_build(const orb_keypoint_t* __restrict__ kps, int n, int minX,
                                                     int minY, float invW, float invH, int* __restrict__ cellStart,
                                                     int* __restrict__ items) {
    // Counting sort in LDS: cell counts, their exclusive scan (wave prefix sums on DPP + the
    // 16 wave totals: 3 barriers instead of round 5's 20-barrier tree), the keypoints placed by
    // LDS cursors, each cell's few entries put back in index order in LDS, the list written out
    // with one coalesced pass (round 5 sorted the cells in global memory: a dependent round trip
    // per entry moved, 18-20 us per call).
    __shared__ int s_cnt[NCELLS];
    __shared__ uint16_t s_items[MAX_TARGET];
    __shared__ int s_wt[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto cell_of = [&](int i) {
        const int px = (int)roundf((kps[i].x - (float)minX) * invW);
        const int py = (int)roundf((kps[i].y - (float)minY) * invH);
        return (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) ? -1 : px * GRID_ROWS + py;
    };
    for (int c = tid; c < NCELLS; c += 1024) s_cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int c = cell_of(i);
        if (c >= 0) atomicAdd(&s_cnt[c], 1);
    }
    __syncthreads();
    const int c0 = tid * 3;  // 3 cells per thread (NCELLS = 3 x 1024)
    const int a = s_cnt[c0], b = s_cnt[c0 + 1], c = s_cnt[c0 + 2];
    const int incl = orbdev::wave_incl_scan(a + b + c);
    if (lane == 63) s_wt[wave] = incl;
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wave; ++w) before += s_wt[w];
    const int base = before + incl - (a + b + c);
    cellStart[c0] = base;
    cellStart[c0 + 1] = base + a;
    cellStart[c0 + 2] = base + a + b;
    int total = 0;
    for (int w = 0; w < 16; ++w) total += s_wt[w];
    if (tid == 0) cellStart[NCELLS] = total;
    s_cnt[c0] = base;  // cursors (each thread its own three cells)
    s_cnt[c0 + 1] = base + a;
    s_cnt[c0 + 2] = base + a + b;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int cc = cell_of(i);
        if (cc >= 0) s_items[atomicAdd(&s_cnt[cc], 1)] = (uint16_t)i;
    }
    __syncthreads();
    // index order inside each of this thread's cells (a handful of entries each)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int s0 = k == 0 ? base : k == 1 ? base + a : base + a + b, e = s_cnt[c0 + k];
        for (int i = s0 + 1; i < e; ++i) {
            const uint16_t v = s_items[i];
            int j = i - 1;
            while (j >= s0 && s_items[j] > v) {
                s_items[j + 1] = s_items[j];
                --j;
            }
            s_items[j + 1] = v;
        }
    }
    __syncthreads();
    for (int i = tid; i < total; i += 1024) items[i] = s_items[i];
}

// ---- k_query_prep ------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_query_prep(Job J) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= J.qn) return;
    const DView& T = J.T;
    QP p;
    p.u = p.v = p.r = 0.f;
    p.flags = 0;
    p.aMin = p.aMax = -1;
    p.pMin = p.pMax = 0;
    p.lo = p.hi = 0;
    const int m = J.mode;
    const int row = qrow(J, q);
    bool ok = true;
    if (m == M_TRIANG)
        ok = !J.qflag[row];  // pMP1 -> continue (ORBmatcher.cc:895-897)
    else if (J.qflag)
        ok = J.qflag[row] != 0;
    if (ok) switch (m) {
            case M_AREA_F:
            case M_AREA_KF:
                p.u = J.qu[q];
                p.v = J.qv[q];
                p.r = J.qvcos[q];
                p.aMin = J.qlevel ? J.qlevel[2 * q] : -1;
                p.aMax = J.qlevel ? J.qlevel[2 * q + 1] : -1;
                p.flags = 1 | (m == M_AREA_KF ? 2 : 0);
                break;
            case M_LOCAL: {  // ORBmatcher.cc:60-74 (+ RadiusByViewingCos 127-133)
                const int pred = J.qlevel[q];
                float r = (double)J.qvcos[q] > 0.998 ? 2.5f : 4.0f;
                if (J.th != 1.0f) r *= J.th;
                p.u = J.qu[q];
                p.v = J.qv[q];
                p.r = r * T.sf[pred];
                p.aMin = pred - 1;
                p.aMax = pred;
                p.flags = 1;
                break;
            }
            case M_WINDOW: {  // 427-446
                const orb_keypoint_t kp1 = J.qkps[q];
                const int level1 = kp1.octave;
                if (J.minLevel > 0 && level1 < J.minLevel) break;
                if (J.maxLevel < INT_MAX && level1 > J.maxLevel) break;
                p.u = kp1.x;
                p.v = kp1.y;
                p.r = (float)J.window;
                p.aMin = p.aMax = level1;
                p.flags = 1;
                break;
            }
            case M_F2F:      // 540-552
            case M_MOTION:   // 1530-1551
            case M_RELOC: {  // 1645-1673
                float X[3];
                gemm3_add(T.R, J.qpos + 3 * q, T.t, X);
                const float xc = X[0], yc = X[1];
                const float invzc = (float)(1.0 / (double)X[2]);
                const float u = __builtin_fmaf(T.fx * xc, invzc, T.cx);
                const float v = __builtin_fmaf(T.fy * yc, invzc, T.cy);
                p.u = u;
                p.v = v;
                if (m == M_F2F) {
                    const int level1 = J.qkps[q].octave;
                    p.r = (float)J.window;
                    p.aMin = p.aMax = level1;
                    p.flags = 1;
                    break;
                }
                if (u < (float)T.minX || u > (float)T.maxX) break;
                if (v < (float)T.minY || v > (float)T.maxY) break;
                if (m == M_MOTION) {
                    const int oct = J.qkps[q].octave;
                    p.r = J.th * T.sf[oct];
                    p.aMin = oct - 1;
                    p.aMax = oct + 1;
                } else {
                    float PO[3];
                    const float* P = J.qpos + 3 * q;
                    PO[0] = P[0] - T.Ow[0];
                    PO[1] = P[1] - T.Ow[1];
                    PO[2] = P[2] - T.Ow[2];
                    const float dist3D = (float)norm3(PO);
                    const float ratio = dist3D / J.qdmin[q];
                    const int pred = predict_level(T, ratio);
                    p.r = J.th * T.sf[pred];
                    p.aMin = pred - 1;
                    p.aMax = pred + 1;
                }
                p.flags = 1;
                break;
            }
            case M_SIM3P:      // 310-366
            case M_FUSE:       // 1038-1089
            case M_FUSE_SCW: {  // 1161-1212
                const float* P = J.qpos + 3 * q;
                float X[3];
                gemm3_add(T.R, P, T.t, X);
                if (X[2] < 0.0f) break;
                const float invz = m == M_FUSE_SCW ? (float)(1.0 / (double)X[2]) : 1.0f / X[2];
                const float x = X[0] * invz, y = X[1] * invz;
                const float u = __builtin_fmaf(T.fx, x, T.cx), v = __builtin_fmaf(T.fy, y, T.cy);
                if (!kf_in_image(T, u, v)) break;
                float PO[3] = {P[0] - T.Ow[0], P[1] - T.Ow[1], P[2] - T.Ow[2]};
                const float dist3D = (float)norm3(PO);
                const float minDistance = J.qdmin[q], maxDistance = J.qdmax[q];
                if (dist3D < minDistance || dist3D > maxDistance) break;
                if (dot3(PO, J.qnormal + 3 * q) < 0.5 * (double)dist3D) break;
                const float ratio = dist3D / minDistance;
                const int pred = predict_level(T, ratio);
                p.u = u;
                p.v = v;
                p.r = J.th * T.sf[pred];
                p.pMin = pred - 1;
                p.pMax = pred;
                p.flags = 1 | 2 | 4;
                break;
            }
            case M_SIM3: {  // 1321-1367 / 1391-1437
                float X1[3], X2[3];
                gemm3_add(J.SRw, J.qpos + 3 * q, J.Stw, X1);
                gemm3_add(J.SR, X1, J.St, X2);
                if (X2[2] < 0.0f) break;
                const float invz = (float)(1.0 / (double)X2[2]);
                const float x = X2[0] * invz, y = X2[1] * invz;
                const float u = __builtin_fmaf(J.qfx, x, J.qcx), v = __builtin_fmaf(J.qfy, y, J.qcy);
                if (!kf_in_image(T, u, v)) break;
                const float dist3D = (float)norm3(X2);
                const float minDistance = J.qdmin[q], maxDistance = J.qdmax[q];
                if (dist3D < minDistance || dist3D > maxDistance) break;
                const float ratio = dist3D / minDistance;
                const int pred = predict_level(T, ratio);
                p.u = u;
                p.v = v;
                p.r = J.th * T.sf[pred];
                p.pMin = pred - 1;
                p.pMax = pred;
                p.flags = 1 | 2 | 4;
                break;
            }
            default: {  // BoW: the FeatureVector merge walk (ORBmatcher.cc:177-262) visits the
                // nodes present in both vectors in ascending id order
                int a = 0, hi = J.fv1N;
                while (a < hi) {  // node of position q: last a with fv1Off[a] <= q
                    const int mid = (a + hi) >> 1;
                    if (J.fv1Off[mid + 1] <= q)
                        a = mid + 1;
                    else
                        hi = mid;
                }
                const uint32_t id = J.fv1Nodes[a];
                int lo2 = 0, hi2 = J.fv2N;
                while (lo2 < hi2) {
                    const int mid = (lo2 + hi2) >> 1;
                    if (J.fv2Nodes[mid] < id)
                        lo2 = mid + 1;
                    else
                        hi2 = mid;
                }
                if (lo2 < J.fv2N && J.fv2Nodes[lo2] == id) {
                    p.lo = J.fv2Off[lo2];
                    p.hi = J.fv2Off[lo2 + 1];
                    p.flags = 1;
                }
                break;
            }
        }
    J.qp[q] = p;
}

// ---- candidate enumeration (one wave, lanes stride the candidates in traversal order) ----
// visit(pos, idx): `pos` is monotone in the reference's candidate order.
template <class V>
__device__ __forceinline__ void enum_candidates(const Job& J, const QP& p, int lane, V&& visit) {
    const DView& T = J.T;
    if (is_bow(J.mode)) {
        for (int pos = p.lo + lane; pos < p.hi; pos += 64) visit(pos, T.items[pos]);
        return;
    }
    // Frame.cc:205-223 / KeyFrame.cc:617-635
    int minCX = (int)floorf((p.u - (float)T.minX - p.r) * T.invW);
    minCX = max(0, minCX);
    if (minCX >= GRID_COLS) return;
    int maxCX = (int)ceilf((p.u - (float)T.minX + p.r) * T.invW);
    maxCX = min(GRID_COLS - 1, maxCX);
    if (maxCX < 0) return;
    int minCY = (int)floorf((p.v - (float)T.minY - p.r) * T.invH);
    minCY = max(0, minCY);
    if (minCY >= GRID_ROWS) return;
    int maxCY = (int)ceilf((p.v - (float)T.minY + p.r) * T.invH);
    maxCY = min(GRID_ROWS - 1, maxCY);
    if (maxCY < 0) return;
    const bool kfArea = p.flags & 2, post = p.flags & 4;
    const bool checkLevels = !(p.aMin == -1 && p.aMax == -1), sameLevel = checkLevels && p.aMin == p.aMax;
    for (int ix = minCX; ix <= maxCX; ++ix) {
        const int lo = T.cellStart[ix * GRID_ROWS + minCY], hi = T.cellStart[ix * GRID_ROWS + maxCY + 1];
        for (int pos = lo + lane; pos < hi; pos += 64) {
            const int idx = T.items[pos];
            const orb_keypoint_t kp = T.kps[idx];
            if (kfArea) {
                if (!(fabsf(kp.x - p.u) <= p.r && fabsf(kp.y - p.v) <= p.r)) continue;
                if (post && (kp.octave < p.pMin || kp.octave > p.pMax)) continue;
            } else {
                if (checkLevels && !sameLevel) {
                    if (kp.octave < p.aMin || kp.octave > p.aMax) continue;
                } else if (sameLevel) {
                    if (kp.octave != p.aMin) continue;
                }
                if (fabsf(kp.x - p.u) > p.r || fabsf(kp.y - p.v) > p.r) continue;
            }
            visit(pos, idx);
        }
    }
}

// Candidate key: (distance << 16) | order; order = traversal position, or the target index
// for SearchForTriangulation (its vDistIndex is sorted by (dist, idx2), ORBmatcher.cc:926).
__device__ __forceinline__ uint32_t cand_key(int mode, int dist, int pos, int idx) {
    return ((uint32_t)dist << 16) | (uint32_t)(mode == M_TRIANG ? idx : pos);
}
__device__ __forceinline__ int key_idx(const Job& J, uint32_t key) {
    return J.mode == M_TRIANG ? (int)(key & 0xFFFF) : J.T.items[key & 0xFFFF];
}

// ---- k_query_scan: one wave per query ---------------------------------------------------
// Each lane keeps its candidates' 8 smallest keys; LK rounds of wave-min merge them into the
// query's LK smallest.  For LK > 8 a lane may own more than 8 of them: once a lane that scanned
// more than 8 candidates has given up its 8th, the later entries are no longer guaranteed, and
// kval[q] records the exact prefix (the resolver rescans past it).
template <int LK>
__global__ void __launch_bounds__(256) k_query_scan(Job J) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (q >= J.qn) return;
    const QP p = J.qp[q];
    int n = 0;
    uint32_t top[TOPK];
#pragma unroll
    for (int k = 0; k < TOPK; ++k) top[k] = 0xFFFFFFFFu;
    if (p.flags & 1) {
        if (J.mode == M_AREA_F || J.mode == M_AREA_KF) {
            enum_candidates(J, p, lane, [&](int, int) { ++n; });
            n = wave_sum(n);
            if (lane == 0) J.cnt[q] = n;
            return;
        }
        uint32_t d1[8];
        load_desc(J.qdesc + (size_t)qrow(J, q) * 8, d1);
        const int m = J.mode;
        enum_candidates(J, p, lane, [&](int pos, int idx) {
            if (J.taken0 && J.taken0[idx]) return;
            if (m == M_BOW_KFKF && !J.tflag[idx]) return;  // !pMP2 || isBad (768-772)
            if (m == M_TRIANG && J.tflag[idx]) return;     // pMP2 (905-907)
            uint32_t d2[8];
            load_desc(J.T.desc + (size_t)idx * 8, d2);
            const int dist = hamming256(d1, d2);
            if (m == M_TRIANG && dist > TH_LOW) return;  // (913-914)
            topk_insert(top, cand_key(m, dist, pos, idx));
            ++n;
        });
    }
    const int nLane = n;
    n = wave_sum(n);
    // merge the lanes' sorted lists: LK rounds of wave-min; keys are unique per candidate
    uint32_t res = 0xFFFFFFFFu;
    int popped = 0, kv = LK;
#pragma unroll
    for (int k = 0; k < LK; ++k) {
        const uint32_t mn = wave_min(top[0]);
        const bool mine = top[0] == mn && mn != 0xFFFFFFFFu;
        if (mine) {
#pragma unroll
            for (int i = 0; i < TOPK - 1; ++i) top[i] = top[i + 1];
            top[TOPK - 1] = 0xFFFFFFFFu;
            ++popped;
        }
        if (lane == k) res = mn;
        if constexpr (LK > TOPK) {
            if (__ballot(mine && popped == TOPK && nLane > TOPK) != 0ull) kv = min(kv, k + 1);
        }
    }
    if (lane < LK) {
        J.topk[(size_t)q * LK + lane] = res;
        // the entry's target and its octave, so the loop-carried resolver reads no dependent
        // global data per query
        uint32_t x = 0;
        if (res != 0xFFFFFFFFu) {
            const int idx = key_idx(J, res);
            x = (uint32_t)idx | ((uint32_t)J.T.kps[idx].octave << 24);
        }
        J.topx[(size_t)q * LK + lane] = x;
    }
    if (lane == 0) {
        J.cnt[q] = n;
        if constexpr (LK > TOPK) J.kval[q] = kv;
    }
}

// AREA: ordered write of every candidate index (wave per query, ballot compaction)
__global__ void __launch_bounds__(256) k_area_fill(Job J) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (q >= J.qn) return;
    const QP p = J.qp[q];
    if (!(p.flags & 1)) return;
    int base = J.areaOff[q];
    // enum_candidates visits in strided lane order; wrap each 64-candidate batch of a cell
    // range with a ballot so the output keeps the traversal order
    const DView& T = J.T;
    int minCX = (int)floorf((p.u - (float)T.minX - p.r) * T.invW);
    minCX = max(0, minCX);
    if (minCX >= GRID_COLS) return;
    int maxCX = (int)ceilf((p.u - (float)T.minX + p.r) * T.invW);
    maxCX = min(GRID_COLS - 1, maxCX);
    if (maxCX < 0) return;
    int minCY = (int)floorf((p.v - (float)T.minY - p.r) * T.invH);
    minCY = max(0, minCY);
    if (minCY >= GRID_ROWS) return;
    int maxCY = (int)ceilf((p.v - (float)T.minY + p.r) * T.invH);
    maxCY = min(GRID_ROWS - 1, maxCY);
    if (maxCY < 0) return;
    const bool kfArea = p.flags & 2;
    const bool checkLevels = !(p.aMin == -1 && p.aMax == -1), sameLevel = checkLevels && p.aMin == p.aMax;
    for (int ix = minCX; ix <= maxCX; ++ix) {
        const int lo = T.cellStart[ix * GRID_ROWS + minCY], hi = T.cellStart[ix * GRID_ROWS + maxCY + 1];
        for (int p0 = lo; p0 < hi; p0 += 64) {
            const int pos = p0 + lane;
            bool keep = false;
            int idx = 0;
            if (pos < hi) {
                idx = T.items[pos];
                const orb_keypoint_t kp = T.kps[idx];
                if (kfArea) {
                    keep = fabsf(kp.x - p.u) <= p.r && fabsf(kp.y - p.v) <= p.r;
                } else {
                    keep = true;
                    if (checkLevels && !sameLevel) {
                        if (kp.octave < p.aMin || kp.octave > p.aMax) keep = false;
                    } else if (sameLevel) {
                        if (kp.octave != p.aMin) keep = false;
                    }
                    if (fabsf(kp.x - p.u) > p.r || fabsf(kp.y - p.v) > p.r) keep = false;
                }
            }
            const uint64_t m = __ballot(keep);
            if (keep) J.areaOut[base + orbdev::lanes_below(m)] = idx;
            base += __popcll(m);
        }
    }
}

// ---- k_resolve -------------------------------------------------------------------------
constexpr int RES_CHUNK = 64;  // queries staged per chunk of the sequential pass
// Exact rescan of query q against the live taken flags: the two smallest keys.
template <class TAKEN>
__device__ void rescan_best2_by(const Job& J, int q, const QP& p, TAKEN&& taken, int lane, uint32_t* b1, uint32_t* b2) {
    uint32_t d1[8];
    load_desc(J.qdesc + (size_t)qrow(J, q) * 8, d1);
    uint32_t lb = 0xFFFFFFFFu, ls = 0xFFFFFFFFu;
    const int m = J.mode;
    enum_candidates(J, p, lane, [&](int pos, int idx) {
        if (taken(idx)) return;
        if (m == M_BOW_KFKF && !J.tflag[idx]) return;
        if (m == M_TRIANG && J.tflag[idx]) return;
        uint32_t d2[8];
        load_desc(J.T.desc + (size_t)idx * 8, d2);
        const int dist = hamming256(d1, d2);
        if (m == M_TRIANG && dist > TH_LOW) return;
        const uint32_t key = cand_key(m, dist, pos, idx);
        if (key < lb) {
            ls = lb;
            lb = key;
        } else if (key < ls) {
            ls = key;
        }
    });
    const uint32_t g1 = wave_min(lb);
    const uint32_t g2 = wave_min(lb == g1 ? ls : lb);
    *b1 = g1;
    *b2 = g2;
}
__device__ void rescan_best2(const Job& J, int q, const QP& p, const uint8_t* s_taken, int lane, uint32_t* b1,
                             uint32_t* b2) {
    rescan_best2_by(J, q, p, [&](int idx) { return s_taken[idx] != 0; }, lane, b1, b2);
}

// SearchForTriangulation rescan: smallest untaken key with dist <= DistTh passing the
// epipolar test (the first such entry of the sorted vDistIndex walk, ORBmatcher.cc:926-955).
__device__ __forceinline__ bool epipolar_ok(const Job& J, const orb_keypoint_t& kp1, const orb_keypoint_t& kp2) {
    // CheckDistEpipolarLine (ORBmatcher.cc:136-153), g++ -O3 -march=native contraction
    const float* F = J.F12;
    const float a = __builtin_fmaf(kp1.x, F[0], kp1.y * F[3]) + F[6];
    const float b = __builtin_fmaf(kp1.x, F[1], kp1.y * F[4]) + F[7];
    const float c = __builtin_fmaf(kp1.y, F[5], kp1.x * F[2]) + F[8];
    const float num = __builtin_fmaf(b, kp2.y, a * kp2.x) + c;
    const float den = __builtin_fmaf(a, a, b * b);
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)J.T.sigma2[kp2.octave];
}

__device__ uint32_t triang_rescan(const Job& J, int q, const QP& p, const uint8_t* s_taken, int lane) {
    uint32_t b1, b2;
    rescan_best2(J, q, p, s_taken, lane, &b1, &b2);
    if (b1 == 0xFFFFFFFFu) return 0xFFFFFFFFu;
    const int distTh = 2 * (int)(b1 >> 16);
    const orb_keypoint_t kp1 = J.qkps[qrow(J, q)];
    uint32_t d1[8];
    load_desc(J.qdesc + (size_t)qrow(J, q) * 8, d1);
    uint32_t best = 0xFFFFFFFFu;
    enum_candidates(J, p, lane, [&](int pos, int idx) {
        if (s_taken[idx] || J.tflag[idx]) return;
        uint32_t d2[8];
        load_desc(J.T.desc + (size_t)idx * 8, d2);
        const int dist = hamming256(d1, d2);
        if (dist > TH_LOW || dist > distTh) return;
        const uint32_t key = cand_key(M_TRIANG, dist, pos, idx);
        if (key < best && epipolar_ok(J, kp1, J.T.kps[idx])) best = key;
    });
    return wave_min(best);
}

// The acceptance test of each matcher for the query's best / second untaken candidates.
template <int MODE>
__device__ __forceinline__ bool accept_rule(const Job& J, int bestDist, int bestDist2, int bestLevel, int bestLevel2) {
    switch (MODE) {
        case M_LOCAL:  // 112-121
            return bestDist <= TH_HIGH && !(bestLevel == bestLevel2 && (float)bestDist > J.nnratio * (float)bestDist2);
        case M_WINDOW:  // 476
        case M_F2F:     // 585
            return (float)bestDist <= (float)bestDist2 * J.nnratio && bestDist <= TH_HIGH;
        case M_BOW_KFF:  // 222-226
            return bestDist <= TH_LOW && (float)bestDist < J.nnratio * (float)bestDist2;
        case M_BOW_KFKF:  // 789-793
            return bestDist < TH_LOW && (float)bestDist < J.nnratio * (float)bestDist2;
        case M_MOTION:  // 1576
            return bestDist <= TH_HIGH;
        case M_RELOC:  // 1701
        case M_SIM3P:  // 393
            return bestDist <= J.thDist;
        case M_TRIANG:
            return true;
        default:
            return false;
    }
}

// One instantiation per matcher (MODE == J.mode): the loop-carried pass of each is its own
// straight-line code, without the other modes' branches.
template <int MODE>
__global__ void __launch_bounds__(256) k_resolve(Job J) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_hist[HISTO + 2];
    __shared__ int s_ind[3];
    __shared__ int s_nacc;
    // the sequential pass's inputs, RES_CHUNK queries per buffer (double-buffered)
    __shared__ int2 s_cq[2][RES_CHUNK];
    __shared__ uint32_t s_ce[2][RES_CHUNK * TOPK], s_cx[2][RES_CHUNK * TOPK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Tn = J.T.n;
    constexpr int m = MODE;
    int* s_out = (int*)smem;                                  // outN
    // accepted matches in acceptance order: (slot << 5) | bin and the partner (the other index of
    // the pair, as accepted: a slot accepted twice keeps both pairs' bins, as rotHist does)
    int* s_acc = s_out + J.outN;                               // Tn (an acceptance takes a target)
    int* s_accp = s_acc + max(Tn, 1);                          // Tn
    uint8_t* s_taken = (uint8_t*)(s_accp + max(Tn, 1));         // Tn
    for (int i = tid; i < J.outN; i += 256) s_out[i] = -1;
    for (int i = tid; i < Tn; i += 256) s_taken[i] = J.taken0 ? J.taken0[i] : 0;
    if (tid == 0) s_nacc = 0;
    __syncthreads();
    const bool rotMode = J.checkOri && (m == M_WINDOW || m == M_MOTION || m == M_RELOC || m == M_BOW_KFF ||
                                        m == M_BOW_KFKF || m == M_TRIANG);
    if (!is_exclusive(m)) {
        // Fuse / SearchBySim3: best distance per query, no cross-query state
        int acc = 0;
        for (int q = tid; q < J.qn; q += 256) {
            if (!(J.qp[q].flags & 1) || J.cnt[q] == 0) continue;
            const uint32_t e = J.topk[(size_t)q * TOPK];
            const int dist = (int)(e >> 16);
            if (dist <= J.thDist) {
                s_out[q] = key_idx(J, e);
                ++acc;
            }
        }
        atomicAdd(&s_nacc, acc);
    } else {
        // A query's inputs (flags, candidate count, top-8 keys with their targets and octaves) do
        // not depend on the loop-carried state: waves 1-3 stage the next RES_CHUNK queries' inputs
        // in LDS (double-buffered, one barrier per chunk) while wave 0 decides the current ones
        // from LDS, so the sequential pass pays LDS round trips per query, no global ones
        int nacc = 0;
        const int nch = (J.qn + RES_CHUNK - 1) / RES_CHUNK;
        auto load_chunk = [&](int c, int buf) {  // waves 1-3
            for (int i = tid - 64; i < RES_CHUNK * TOPK; i += 192) {
                const int q = c * RES_CHUNK + (i >> 3);
                s_ce[buf][i] = q < J.qn ? J.topk[(size_t)q * TOPK + (i & 7)] : 0xFFFFFFFFu;
                s_cx[buf][i] = q < J.qn ? J.topx[(size_t)q * TOPK + (i & 7)] : 0u;
            }
            for (int i = tid - 64; i < RES_CHUNK; i += 192) {
                const int q = c * RES_CHUNK + i;
                s_cq[buf][i] = q < J.qn ? make_int2(J.qp[q].flags, J.cnt[q]) : make_int2(0, 0);
            }
        };
        if (wave != 0 && nch > 0) load_chunk(0, 0);
        __syncthreads();
        for (int c = 0; c < nch; ++c) {
            if (wave != 0) {
                if (c + 1 < nch) load_chunk(c + 1, (c + 1) & 1);
            } else {
                const int buf = c & 1, qend = min(RES_CHUNK, J.qn - c * RES_CHUNK);
                // one query decided exactly (the triangulation walk, a query whose top-8 ran out)
                auto single = [&](int jq) {
                    const int q = c * RES_CHUNK + jq;
                    const int2 fc = s_cq[buf][jq];
                    const int flags = __builtin_amdgcn_readfirstlane(fc.x), cnt = __builtin_amdgcn_readfirstlane(fc.y);
                    if (!(flags & 1)) return;
                    if (cnt == 0) return;
                    const uint32_t eL = lane < TOPK ? s_ce[buf][jq * TOPK + lane] : 0xFFFFFFFFu;
                    const uint32_t xL = lane < TOPK ? s_cx[buf][jq * TOPK + lane] : 0u;
                    const int k = min(cnt, TOPK);
                    const uint32_t e = lane < k ? eL : 0xFFFFFFFFu;
                    const int eidx = lane < k ? (int)(xL & 0xFFFFFFu) : 0;
                    const bool untaken = lane < k && !s_taken[eidx];
                    const uint64_t um = __ballot(untaken);
                    int bestIdx = -1, bestDist = INT_MAX, bestDist2 = INT_MAX, bestLevel = -1, bestLevel2 = -1;
                    if (m == M_TRIANG) {
                        // walk the sorted list: BestDist from the first untaken entry, then the first
                        // untaken entry within round(2*BestDist) that passes the epipolar test
                        uint32_t chosen = 0xFFFFFFFFu;
                        bool decided = false;
                        if (um != 0ull) {
                            const int first = __ffsll((unsigned long long)um) - 1;
                            const int distTh = 2 * (int)((uint32_t)__builtin_amdgcn_readlane((int)e, first) >> 16);
                            const orb_keypoint_t kp1 = J.qkps[qrow(J, q)];
                            const bool inTh = lane < k && (int)(e >> 16) <= distTh;  // (epipolar: the target's point, below)
                            const bool pass = untaken && inTh && epipolar_ok(J, kp1, J.T.kps[eidx]);
                            const uint64_t pm = __ballot(pass), om = __ballot(lane < k && !inTh);
                            if (pm != 0ull) {
                                chosen = (uint32_t)__builtin_amdgcn_readlane((int)e, __ffsll((unsigned long long)pm) - 1);
                                decided = true;
                            } else if (om != 0ull || cnt <= TOPK) {
                                decided = true;  // the walk breaks on an entry past DistTh, or ends
                            }
                        } else if (cnt <= TOPK) {
                            decided = true;
                        }
                        if (!decided) chosen = triang_rescan(J, q, J.qp[q], s_taken, lane);
                        if (chosen == 0xFFFFFFFFu) return;
                        bestIdx = key_idx(J, chosen);
                        bestDist = 0;  // accepted below unconditionally
                    } else {
                        const int need = needs_second(m) ? 2 : 1;
                        uint32_t b1 = 0xFFFFFFFFu, b2 = 0xFFFFFFFFu;
                        uint32_t x1 = 0u, x2 = 0u;
                        if (__popcll(um) >= need || cnt <= TOPK) {
                            if (um != 0ull) {
                                // (wave-uniform lanes: v_readlane, no LDS round trip)
                                const int l1 = __ffsll((unsigned long long)um) - 1;
                                b1 = (uint32_t)__builtin_amdgcn_readlane((int)e, l1);
                                x1 = (uint32_t)__builtin_amdgcn_readlane((int)xL, l1);
                                const uint64_t um2 = um & (um - 1);
                                if (um2) {
                                    const int l2 = __ffsll((unsigned long long)um2) - 1;
                                    b2 = (uint32_t)__builtin_amdgcn_readlane((int)e, l2);
                                    x2 = (uint32_t)__builtin_amdgcn_readlane((int)xL, l2);
                                }
                            }
                        } else {
                            rescan_best2(J, q, J.qp[q], s_taken, lane, &b1, &b2);
                            if (b1 != 0xFFFFFFFFu) {
                                const int i1x = key_idx(J, b1);
                                x1 = (uint32_t)i1x | ((uint32_t)J.T.kps[i1x].octave << 24);
                            }
                            if (b2 != 0xFFFFFFFFu) {
                                const int i2x = key_idx(J, b2);
                                x2 = (uint32_t)i2x | ((uint32_t)J.T.kps[i2x].octave << 24);
                            }
                        }
                        if (b1 == 0xFFFFFFFFu) return;  // every candidate taken: bestDist stays INT_MAX
                        bestIdx = (int)(x1 & 0xFFFFFFu);
                        bestDist = (int)(b1 >> 16);
                        bestLevel = (int)(x1 >> 24);
                        if (b2 != 0xFFFFFFFFu) {
                            bestDist2 = (int)(b2 >> 16);
                            bestLevel2 = (int)(x2 >> 24);
                        }
                    }
                    const bool accept = accept_rule<m>(J, bestDist, bestDist2, bestLevel, bestLevel2);
                    if (!accept) return;
                    if (lane == 0) {
                        s_taken[bestIdx] = 1;
                        const int qv = qrow(J, q);
                        const int slot = J.outByTarget ? bestIdx : qv;
                        s_out[slot] = J.outByTarget ? qv : bestIdx;
                        if (rotMode) {  // its rotation bin: after the pass, in parallel
                            s_acc[nacc] = slot << 5;
                            s_accp[nacc] = J.outByTarget ? qv : bestIdx;
                        }
                    }
                    ++nacc;
                    // lane 0's LDS writes land before any lane's next read (same wave, in order)
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                };
                if constexpr (m == M_TRIANG) {
                    for (int jq = 0; jq < qend; ++jq) single(jq);
                } else {
                    // Speculated eight queries at a time (lane 8g + k: query jq + g, entry k of its
                    // sorted top-8), as k_match_init's greedy pass: a query's outcome is fixed by its
                    // first two untaken entries (best, second) and an acceptance takes exactly one
                    // target, so every query of the batch is decided from the batch-start state
                    // unless an earlier query of the batch accepted its best or second target, or it
                    // needs the exact rescan (a truncated top-8 with too few untaken entries); the
                    // batch commits its queries before the first such one.
                    const int grp = lane >> 3, cand = lane & 7;
                    const int need = needs_second(m) ? 2 : 1;
                    int jq = 0;
                    while (jq < qend) {
                        const int nb = min(8, qend - jq);
                        const int jg = jq + min(grp, nb - 1);
                        const int2 fc = s_cq[buf][jg];
                        const uint32_t eR = s_ce[buf][jg * TOPK + cand];
                        const uint32_t xR = s_cx[buf][jg * TOPK + cand];
                        const bool qok = grp < nb && (fc.x & 1) && fc.y > 0;
                        const int cnt = qok ? fc.y : 0;
                        const bool valid = cand < min(cnt, TOPK);
                        const int idx = (int)(xR & 0xFFFFFFu);
                        const bool untaken = valid && !s_taken[idx];
                        const uint32_t best = min8(untaken ? eR : 0xFFFFFFFFu);
                        const bool isB = untaken && eR == best;
                        const uint32_t sec = min8(untaken && !isB ? eR : 0xFFFFFFFFu);
                        const bool isS = untaken && eR == sec;
                        // the targets (and octaves) of best and second, to every lane of the group
                        const uint32_t tB = min8(isB ? xR : 0xFFFFFFFFu), tS = min8(isS ? xR : 0xFFFFFFFFu);
                        const uint64_t um = __ballot(untaken);
                        const int nUnt = __popcll((um >> (8 * grp)) & 0xFFull);
                        const bool rescan = qok && cnt > TOPK && nUnt < need;
                        bool accept = false;
                        if (qok && !rescan && best != 0xFFFFFFFFu) {
                            const int bestDist = (int)(best >> 16), bestLevel = (int)(tB >> 24);
                            const int bestDist2 = sec != 0xFFFFFFFFu ? (int)(sec >> 16) : INT_MAX;
                            const int bestLevel2 = sec != 0xFFFFFFFFu ? (int)(tS >> 24) : -1;
                            accept = accept_rule<m>(J, bestDist, bestDist2, bestLevel, bestLevel2);
                        }
                        const int bIdx = (int)(tB & 0xFFFFFFu), sIdx = sec != 0xFFFFFFFFu ? (int)(tS & 0xFFFFFFu) : -1;
                        // bit g: group g accepts
                        const uint64_t accW = __ballot(accept && cand == 0);
                        // lane 8g + k checks group k's accepted target against query g's best / second
                        const int bIdxK = __shfl(bIdx, 8 * cand, 64);
                        // (best-only matchers: the second does not decide, so only the best can be hit)
                        // KF-KF over a non-unique FeatureVector: two queries of the batch may be one
                        // keypoint row (output slot); the later one must see the earlier's commit
                        bool sameRow = false;
                        if constexpr (m == M_BOW_KFKF) {
                            const int qvG = qrow(J, c * RES_CHUNK + jg);
                            sameRow = __shfl(qvG, 8 * cand, 64) == qvG;
                        }
                        const bool hit = cand < grp && ((accW >> (8 * cand)) & 1ull) &&
                                         (bIdxK == bIdx || (need == 2 && bIdxK == sIdx) || sameRow);
                        const uint64_t stopM = __ballot(grp < nb && (hit || (rescan && cand == 0)));
                        const int jstop = stopM ? (__ffsll((unsigned long long)stopM) - 1) >> 3 : nb;
                        if (accept && cand == 0 && grp < jstop) {
                            // distinct targets (no hit before jstop): these writes commute
                            s_taken[bIdx] = 1;
                            const int qv = qrow(J, c * RES_CHUNK + jg);
                            const int slot = J.outByTarget ? bIdx : qv;
                            s_out[slot] = J.outByTarget ? qv : bIdx;
                            if (rotMode) {
                                // rank among the batch's committed acceptances: query order kept
                                const uint64_t before = accW & ((1ull << (8 * grp)) - 1ull);
                                s_acc[nacc + __popcll(before)] = slot << 5;
                                s_accp[nacc + __popcll(before)] = J.outByTarget ? qv : bIdx;
                            }
                        }
                        nacc += __popcll(accW & (jstop >= 8 ? ~0ull : ((1ull << (8 * jstop)) - 1ull)));
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if (jstop > 0) {
                            jq += jstop;
                        } else {
                            single(jq);  // query jq needs the exact rescan
                            jq += 1;
                        }
                    }
                }
            }
            __syncthreads();  // chunk c decided, chunk c + 1 staged
        }
        if (wave == 0 && lane == 0) s_nacc = nacc;
    }
    __syncthreads();
    int removed = 0;
    if (rotMode && is_exclusive(m)) {  // rotation consistency (e.g. ORBmatcher.cc:491-512)
        const int nacc = s_nacc;
        if (tid < HISTO) s_hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < nacc; i += 256) {
            const int slot = s_acc[i] >> 5, v = s_accp[i];
            const int qv = J.outByTarget ? v : slot, ti = J.outByTarget ? slot : v;
            const int bin = rot_bin(J.qkps[qv].angle, J.T.kps[ti].angle);
            s_acc[i] = (slot << 5) | bin;
            atomicAdd(&s_hist[bin], 1);
        }
        __syncthreads();
        if (tid == 0) {  // ComputeThreeMaxima (1748-1789)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO; ++i) {
                const int sz = s_hist[i];
                if (sz > max1) {
                    max3 = max2;
                    max2 = max1;
                    max1 = sz;
                    ind3 = ind2;
                    ind2 = ind1;
                    ind1 = i;
                } else if (sz > max2) {
                    max3 = max2;
                    max2 = sz;
                    ind3 = ind2;
                    ind2 = i;
                } else if (sz > max3) {
                    max3 = sz;
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
        for (int i = tid; i < nacc; i += 256) {
            const int b = s_acc[i] & 31;
            if (b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) {
                s_out[s_acc[i] >> 5] = -1;
                ++removed;
            }
        }
    }
    removed = wave_sum(removed);
    __syncthreads();
    if (lane == 0 && removed) atomicAdd(&s_nacc, -removed);
    __syncthreads();
    for (int i = tid; i < J.outN; i += 256) J.out[i] = s_out[i];
    if (tid == 0) J.nOut[0] = s_nacc;
}

// The projection-family matchers without a sequential pass: SearchByProjection (local map,
// ORBmatcher.cc:49-125; motion 1507-1620; relocalisation 1622-1746; Sim3 286-407; frame to
// frame 519-594) and WindowSearch (409-516).  A query's decision is a function of which of its
// candidates earlier queries took (e.g. `F.mvpMapPoints[idx]` set earlier in the loop,
// ORBmatcher.cc:87-88): with takenBy[t] = the smallest query that
// accepted target t (-1: taken before the call), query q sees t taken iff takenBy[t] < q.  Every
// query is decided in parallel from the previous iteration's takenBy, the accepted targets give
// the next takenBy (atomicMin), until takenBy repeats.  The sequential result is the unique
// fixed point (query q depends only on queries < q, so by induction on q any fixed point equals
// it) and the iteration reaches it: after iteration k queries 0 .. k-1 are final, and it stops
// as soon as nothing changes (a handful of iterations: a decision changes only when an earlier
// query's acceptance takes its best or second candidate).  A query whose top-8 holds too few
// untaken entries is rescanned exactly (one wave, k_resolve's rescan with this predicate).
// The loop is bounded by qn + 2 iterations (the induction's bound + the one that sees no
// change); past it the kernel reports -1 matches and the call fails (cannot happen).
#define RF_THREADS 1024
#ifndef RF_DEBUG
#define RF_DEBUG 0  // 1: iterations / rescans per call printed (experiment builds)
#endif
#ifndef RF_LONG_LISTS
#define RF_LONG_LISTS 1  // 32-entry lists for the fixed-point resolver except SearchByProjection(local)
#endif
#ifndef RF_ALL_MODES
#define RF_ALL_MODES 1  // 0: the fixed point for SearchByProjection(local) only
#endif
size_t resolve_fix_lds(const Job& J) { return (size_t)2 * std::max(J.T.n, 1) * 4 + (size_t)std::max(J.qn, 1) * 4 + 16; }
template <int MODE>
__global__ void __launch_bounds__(RF_THREADS) k_resolve_fix(Job J) {
    // the projection-family matchers whose only loop-carried state is the taken targets (each
    // reports by target: out[target] = query)
    static_assert(MODE == M_LOCAL || MODE == M_WINDOW || MODE == M_F2F || MODE == M_MOTION || MODE == M_RELOC ||
                      MODE == M_SIM3P,
                  "fixed-point resolver mode");
    extern __shared__ __attribute__((aligned(16))) int rsm[];
    __shared__ int s_changed, s_nres, s_nacc;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Tn = J.T.n;
    int* s_tb = rsm;                  // takenBy, this iteration's input
    int* s_tn = s_tb + max(Tn, 1);    // next iteration's
    int* s_res = s_tn + max(Tn, 1);   // queries needing the exact rescan
    for (int t = tid; t < Tn; t += RF_THREADS) s_tb[t] = J.taken0 && J.taken0[t] ? -1 : INT_MAX;
    constexpr int need = needs_second(MODE) ? 2 : 1;
    bool done = false;
#if RF_DEBUG
    int dbgIt = 0, dbgRes = 0;
#endif
    for (int it = 0; it < J.qn + 2 && !done; ++it) {
#if RF_DEBUG
        ++dbgIt;
#endif
        for (int t = tid; t < Tn; t += RF_THREADS) s_tn[t] = J.taken0 && J.taken0[t] ? -1 : INT_MAX;
        if (tid == 0) {
            s_nres = 0;
            s_changed = 0;
        }
        __syncthreads();
        for (int q = tid; q < J.qn; q += RF_THREADS) {
            if (!(J.qp[q].flags & 1)) continue;
            const int cnt = J.cnt[q];
            if (cnt == 0) continue;
            const int kv = J.topS == TOPK_FIX ? J.kval[q] : TOPK;  // the list's exact prefix
            const int k = min(cnt, kv);
            uint32_t b1 = 0xFFFFFFFFu, b2 = 0xFFFFFFFFu, x1 = 0u, x2 = 0u;
            int nUnt = 0;
            for (int j = 0; j < k; ++j) {
                const uint32_t x = J.topx[(size_t)q * J.topS + j];
                if (s_tb[x & 0xFFFFFFu] < q) continue;
                const uint32_t e = J.topk[(size_t)q * J.topS + j];
                if (nUnt == 0) {
                    b1 = e;
                    x1 = x;
                } else if (nUnt == 1) {
                    b2 = e;
                    x2 = x;
                }
                if (++nUnt == need) break;
            }
            if (cnt > k && nUnt < need) {
                s_res[atomicAdd(&s_nres, 1)] = q;
                continue;
            }
            if (b1 == 0xFFFFFFFFu) continue;
            const int bestDist2 = b2 != 0xFFFFFFFFu ? (int)(b2 >> 16) : INT_MAX;
            const int bestLevel2 = b2 != 0xFFFFFFFFu ? (int)(x2 >> 24) : -1;
            if (accept_rule<MODE>(J, (int)(b1 >> 16), bestDist2, (int)(x1 >> 24), bestLevel2))
                atomicMin(&s_tn[x1 & 0xFFFFFFu], q);
        }
        __syncthreads();
#if RF_DEBUG
        dbgRes += s_nres;
#endif
        for (int r = wave; r < s_nres; r += RF_THREADS / 64) {  // exact rescans, a wave each
            const int q = s_res[r];
            uint32_t b1, b2;
            rescan_best2_by(J, q, J.qp[q], [&](int idx) { return s_tb[idx] < q; }, lane, &b1, &b2);
            if (b1 == 0xFFFFFFFFu) continue;
            const int i1 = key_idx(J, b1);
            const int l1 = J.T.kps[i1].octave;
            const int bestDist2 = b2 != 0xFFFFFFFFu ? (int)(b2 >> 16) : INT_MAX;
            const int bestLevel2 = b2 != 0xFFFFFFFFu ? J.T.kps[key_idx(J, b2)].octave : -1;
            if (lane == 0 && accept_rule<MODE>(J, (int)(b1 >> 16), bestDist2, l1, bestLevel2)) atomicMin(&s_tn[i1], q);
        }
        __syncthreads();
        bool ch = false;
        for (int t = tid; t < Tn; t += RF_THREADS) {
            ch |= s_tn[t] != s_tb[t];
            s_tb[t] = s_tn[t];
        }
        if (ch) s_changed = 1;
        __syncthreads();
        done = s_changed == 0;
        __syncthreads();  // s_changed read by all before the next iteration resets it
    }
    // the rotation consistency check of the matchers that have one (e.g. ORBmatcher.cc:491-512):
    // the histogram counts every final acceptance, order-free
    __shared__ int s_hist[HISTO + 2];
    __shared__ int s_ind[3];
    const bool rotMode = J.checkOri && (MODE == M_WINDOW || MODE == M_MOTION || MODE == M_RELOC);
    if (tid == 0) s_nacc = 0;
    if (rotMode) {
        if (tid < HISTO) s_hist[tid] = 0;
        __syncthreads();
        for (int t = tid; t < Tn; t += RF_THREADS) {
            const int v = s_tb[t];
            if (v >= 0 && v != INT_MAX) atomicAdd(&s_hist[rot_bin(J.qkps[qrow(J, v)].angle, J.T.kps[t].angle)], 1);
        }
        __syncthreads();
        if (tid == 0) {  // ComputeThreeMaxima (1748-1789)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO; ++i) {
                const int sz = s_hist[i];
                if (sz > max1) {
                    max3 = max2;
                    max2 = max1;
                    max1 = sz;
                    ind3 = ind2;
                    ind2 = ind1;
                    ind1 = i;
                } else if (sz > max2) {
                    max3 = max2;
                    max2 = sz;
                    ind3 = ind2;
                    ind2 = i;
                } else if (sz > max3) {
                    max3 = sz;
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
    }
    __syncthreads();
    int acc = 0;
    for (int t = tid; t < J.outN; t += RF_THREADS) {  // outN == Tn (by target)
        const int v = s_tb[t];
        bool a = v >= 0 && v != INT_MAX;
        if (a && rotMode) {
            const int bn = rot_bin(J.qkps[qrow(J, v)].angle, J.T.kps[t].angle);
            a = bn == s_ind[0] || bn == s_ind[1] || bn == s_ind[2];
        }
        J.out[t] = a ? qrow(J, v) : -1;
        acc += a;
    }
    acc = wave_sum(acc);
    if (lane == 0 && acc) atomicAdd(&s_nacc, acc);
    __syncthreads();
    if (tid == 0) {
        J.nOut[0] = done ? s_nacc : -1;
#if RF_DEBUG
        printf("k_resolve_fix mode %d qn %d Tn %d: %d iterations, %d rescans, %d accepted\n", MODE, J.qn, Tn, dbgIt,
               dbgRes, s_nacc);
#endif
    }
}

// SearchBySim3 agreement (ORBmatcher.cc:1489-1502): match12[i1] = idx2 iff vnMatch2[idx2] == i1.
__global__ void k_sim3_agree(const int* __restrict__ m1, int n1, const int* __restrict__ m2, int* __restrict__ out,
                             int* __restrict__ nOut) {
    __shared__ int s_n;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    int c = 0;
    for (int i = threadIdx.x; i < n1; i += blockDim.x) {
        const int idx2 = m1[i];
        const bool ok = idx2 >= 0 && m2[idx2] == i;
        out[i] = ok ? idx2 : -1;
        c += ok;
    }
    atomicAdd(&s_n, c);
    __syncthreads();
    if (threadIdx.x == 0) nOut[0] = s_n;
}

// =========================================================================================
// host side
// =========================================================================================
int fail(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }

}  // namespace

// ---- per-thread host contexts (orb_internal.h) -------------------------------------------
int OrbHostCtx::reserve(size_t dev_bytes, size_t host_bytes) {
    if (!stream) {
        hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
        if (e != hipSuccess) return orb_internal_set_error(ORB_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    if (dev_bytes > cap) {
        const size_t want = std::max(dev_bytes, cap * 2);
        if (buf) (void)hipFree(buf);
        buf = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&buf, want);
        if (e != hipSuccess) return orb_internal_set_error(ORB_EDEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
        cap = want;
    }
    if (host_bytes > pcap) {
        const size_t want = std::max(host_bytes, pcap * 2);
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
        pcap = 0;
        hipError_t e = hipHostMalloc((void**)&pinned, want, hipHostMallocDefault);
        if (e != hipSuccess) return orb_internal_set_error(ORB_EDEVICE, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        pcap = want;
    }
    return ORB_OK;
}

namespace {
// Contexts are never destroyed (no HIP teardown at exit); a thread's contexts go back to the
// pool when it exits.
struct CtxPool {
    std::mutex mu;
    std::vector<OrbHostCtx*> free[64];
};
CtxPool& ctx_pool() {
    static CtxPool* p = new CtxPool();
    return *p;
}
struct ThreadCtxs {
    OrbHostCtx* c[64] = {};
    ~ThreadCtxs() {
        CtxPool& P = ctx_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        for (int d = 0; d < 64; ++d)
            if (c[d]) P.free[d].push_back(c[d]);
    }
};
thread_local ThreadCtxs t_ctxs;
}  // namespace

OrbHostCtx* orb_internal_thread_ctx(int device) {
    if (device < 0 || device >= 64) return nullptr;
    OrbHostCtx*& c = t_ctxs.c[device];
    if (!c) {
        CtxPool& P = ctx_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        if (!P.free[device].empty()) {
            c = P.free[device].back();
            P.free[device].pop_back();
        } else {
            c = new OrbHostCtx();
            c->device = device;
        }
    }
    return c;
}

namespace {
// Bump allocator over one device buffer; `stage` copies a host array into it.
// The staged inputs of a call, copied into the arena by a kernel reading the pinned staging
// (mapped host memory) directly: in-stream with the call's kernels, so no copy-engine hand-off
// (the SDMA copy of ~100 KB took 8.5 us plus ~8 us until the first kernel started, rocprofv3
// timeline of build/latency_gpu, profiles/r06/).  16-B units, a grid-stride loop.
__global__ void __launch_bounds__(256) k_stage_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16,
                                                    const uint8_t* __restrict__ srcb, uint8_t* __restrict__ dstb,
                                                    int tail) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail) dstb[threadIdx.x] = srcb[threadIdx.x];
}
#define STAGE_KERNEL_MAX (8u << 20)  // larger uploads take the copy engine
// The results of a call, copied from the arena into the pinned staging by one workgroup that
// then publishes a completion flag (system-scope release, as k_match_init's host call): the
// host spins on the flag instead of a D2H copy command plus a stream synchronisation.
__global__ void __launch_bounds__(256) k_stage_out(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                   int bytes, int* __restrict__ flag, int seq) {
    const int n16 = bytes >> 4;
    for (int i = threadIdx.x; i < n16; i += 256) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    if ((int)threadIdx.x < (bytes & 15)) dst[(n16 << 4) + threadIdx.x] = src[(n16 << 4) + threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
#define STAGE_OUT_MAX (256u << 10)  // larger results take a D2H copy + stream synchronisation

struct Arena {
    std::vector<std::pair<size_t, std::pair<const void*, size_t>>> uploads;
    size_t size = 0;
    size_t take(size_t bytes) {
        const size_t off = size;
        size += (bytes + 255) & ~(size_t)255;
        return off;
    }
    size_t stage(const void* host, size_t bytes) {
        const size_t off = take(bytes ? bytes : 1);
        if (host && bytes) uploads.push_back({off, {host, bytes}});
        return off;
    }
    void put(size_t off, const void* host, size_t bytes) {  // into a region from take()
        if (host && bytes) uploads.push_back({off, {host, bytes}});
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        hipGetDevice(&prev);
        hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// A call in flight: the arena layout is planned first (offsets), then allocated + uploaded.
struct Call {
    int device;
    OrbHostCtx* ctx = nullptr;
    Arena A;
    uint8_t* base = nullptr;
    template <class T>
    T* at(size_t off) const {
        return (T*)(base + off);
    }
    int begin() {
        if (device < 0 || device >= 64) return fail(ORB_EINVAL, "bad device ordinal");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device >= n) return fail(ORB_EINVAL, "no such HIP device");
        ctx = orb_internal_thread_ctx(device);
        return ORB_OK;
    }
    // allocate (grow) the arena and upload every staged array in one H2D copy
    std::vector<std::pair<void*, std::pair<size_t, size_t>>> pending;  // (host, (off, bytes)) downloads
    bool inflight = false;  // work queued on ctx->stream since the last sync()
    size_t flagOff = 0;  // the completion flag's offset in the staging (past the arena's)
    int commit() {
        flagOff = (A.size + 255) & ~(size_t)255;
        if (int st = ctx->reserve(A.size, flagOff + 256)) return st;
        inflight = true;
        base = ctx->buf;
        size_t hi = 0;
        for (auto& u : A.uploads) {
            std::memcpy(ctx->pinned + u.first, u.second.first, u.second.second);
            hi = std::max(hi, u.first + u.second.second);
        }
        if (hi && hi <= STAGE_KERNEL_MAX) {
            const size_t n16 = hi >> 4;
            const int tail = (int)(hi & 15);
            const unsigned grid = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (n16 + 255) / 256));
            hipLaunchKernelGGL(k_stage_copy, dim3(grid), dim3(256), 0, ctx->stream, (uint4*)base,
                               (const uint4*)ctx->pinned, n16, ctx->pinned + (n16 << 4), base + (n16 << 4), tail);
            HIPCHK(hipGetLastError());
        } else if (hi) {
            HIPCHK(hipMemcpyAsync(base, ctx->pinned, hi, hipMemcpyHostToDevice, ctx->stream));
        }
        return ORB_OK;
    }
    // D2H through the pinned staging (the arena offset is also the staging offset): download()
    // records a region, sync() copies the span of all recorded regions in ONE D2H copy (results
    // are taken last and lie together: a copy costs ~5 us of latency, the bytes between them
    // nothing) and then fills the callers' buffers
    int download(void* host, size_t off, size_t bytes) {
        inflight = true;
        if (bytes) pending.push_back({host, {off, bytes}});
        return ORB_OK;
    }
    int sync() {
        bool seen = false;
        if (!pending.empty()) {
            size_t lo = pending[0].second.first, hi = lo;
            for (auto& d : pending) {
                lo = std::min(lo, d.second.first);
                hi = std::max(hi, d.second.first + d.second.second);
            }
            if (hi - lo <= STAGE_OUT_MAX) {
                static thread_local int seq = 0;
                seq = seq == 0x7fffffff ? 1 : seq + 1;
                volatile int* flag = (volatile int*)(ctx->pinned + flagOff);
                *flag = 0;
                hipLaunchKernelGGL(k_stage_out, dim3(1), dim3(256), 0, ctx->stream, ctx->pinned + lo, base + lo,
                                   (int)(hi - lo), (int*)(ctx->pinned + flagOff), seq);
                HIPCHK(hipGetLastError());
                const auto t0 = std::chrono::steady_clock::now();
                for (int spin = 0;; ++spin) {
                    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) {
                        seen = true;
                        break;
                    }
                    if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
                }
            } else {
                HIPCHK(hipMemcpyAsync(ctx->pinned + lo, base + lo, hi - lo, hipMemcpyDeviceToHost, ctx->stream));
            }
        }
        // (the flag is the kernel's last write, nothing of the call runs after it; without it --
        // no results, an error, a call past the bound -- the stream is synchronised)
        if (!seen) HIPCHK(hipStreamSynchronize(ctx->stream));
        inflight = false;
        for (auto& d : pending) std::memcpy(d.first, ctx->pinned + d.second.first, d.second.second);
        pending.clear();
        return ORB_OK;
    }
    // an early error return leaves work queued on the context's stream: drain it so the next
    // call on this thread can reuse the arena and the staging
    ~Call() {
        if (inflight) (void)hipStreamSynchronize(ctx->stream);
    }
};

int check_view(const orb_frame_view_t* v, const char* name) {
    if (!v) return fail(ORB_EINVAL, std::string(name) + ": NULL view");
    if (v->n < 0 || v->n > MAX_TARGET) return fail(ORB_ENOTSUP, std::string(name) + ": keypoint count out of range");
    if (v->n > 0 && (!v->kps || !v->desc)) return fail(ORB_EINVAL, std::string(name) + ": NULL keypoints/descriptors");
    if (v->nlevels < 1 || v->nlevels > ORB_MAX_VIEW_LEVELS)
        return fail(ORB_EINVAL, std::string(name) + ": nlevels out of range");
    if (v->bounds.max_x <= v->bounds.min_x || v->bounds.max_y <= v->bounds.min_y)
        return fail(ORB_EINVAL, std::string(name) + ": bad bounds");
    for (int i = 0; i < v->n; ++i)
        if (v->kps[i].octave < 0 || v->kps[i].octave >= v->nlevels)
            return fail(ORB_EINVAL, std::string(name) + ": keypoint octave out of range");
    return ORB_OK;
}

// Offsets of a target view inside the arena.
struct ViewOffs {
    size_t kps, desc, cellStart, items;
};

ViewOffs plan_view(Arena& A, const orb_frame_view_t* v, bool grid) {
    ViewOffs o{};
    o.kps = A.stage(v->kps, (size_t)v->n * sizeof(orb_keypoint_t));
    o.desc = A.stage(v->desc, (size_t)v->n * 32);
    if (grid) {
        o.cellStart = A.take((NCELLS + 1) * sizeof(int));
        o.items = A.take((size_t)std::max(v->n, 1) * sizeof(int));
    }
    return o;
}

DView make_dview(const Call& C, const orb_frame_view_t* v, const ViewOffs& o, bool grid) {
    DView d{};
    d.kps = C.at<orb_keypoint_t>(o.kps);
    d.desc = C.at<uint32_t>(o.desc);
    d.n = v->n;
    d.nlevels = v->nlevels;
    d.minX = v->bounds.min_x;
    d.maxX = v->bounds.max_x;
    d.minY = v->bounds.min_y;
    d.maxY = v->bounds.max_y;
    d.invW = static_cast<float>(GRID_COLS) / static_cast<float>(v->bounds.max_x - v->bounds.min_x);
    d.invH = static_cast<float>(GRID_ROWS) / static_cast<float>(v->bounds.max_y - v->bounds.min_y);
    std::memcpy(d.sf, v->scale_factors, sizeof(d.sf));
    std::memcpy(d.sigma2, v->level_sigma2, sizeof(d.sigma2));
    d.fx = v->fx;
    d.fy = v->fy;
    d.cx = v->cx;
    d.cy = v->cy;
    std::memcpy(d.R, v->Rcw, sizeof(d.R));
    std::memcpy(d.t, v->tcw, sizeof(d.t));
    std::memcpy(d.Ow, v->Ow, sizeof(d.Ow));
    if (grid) {
        d.cellStart = C.at<int>(o.cellStart);
        d.items = C.at<int>(o.items);
    }
    return d;
}

int launch_grid(const Call& C, const DView& d) {
    hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), 0, C.ctx->stream, d.kps, d.n, d.minX, d.minY, d.invW,
                       d.invH, (int*)d.cellStart, (int*)d.items);
    HIPCHK(hipGetLastError());
    return ORB_OK;
}

// Scratch of a job: qp, topk, cnt (+ outputs).
struct JobOffs {
    size_t qp, topk, topx, kval, cnt, out, nOut;
};
JobOffs plan_job(Arena& A, int qn, int outN) {
    JobOffs o{};
    o.qp = A.take((size_t)std::max(qn, 1) * sizeof(QP));
    o.topk = A.take((size_t)std::max(qn, 1) * TOPK_FIX * 4);
    o.topx = A.take((size_t)std::max(qn, 1) * TOPK_FIX * 4);
    o.kval = A.take((size_t)std::max(qn, 1) * 4);
    o.cnt = A.take((size_t)std::max(qn, 1) * 4);
    o.out = A.take((size_t)std::max(outN, 1) * 4);
    o.nOut = A.take(16);
    return o;
}
void bind_job(const Call& C, Job& J, const JobOffs& o, int qn, int outN) {
    J.qn = qn;
    J.qp = C.at<QP>(o.qp);
    J.topk = C.at<uint32_t>(o.topk);
    J.topx = C.at<uint32_t>(o.topx);
    J.kval = C.at<int>(o.kval);
    J.topS = TOPK;
    J.cnt = C.at<int>(o.cnt);
    J.out = C.at<int>(o.out);
    J.outN = outN;
    J.nOut = C.at<int>(o.nOut);
}

int resolve_lds(const Job& J, size_t* bytes) {
    *bytes = (size_t)J.outN * 4 + (size_t)std::max(J.T.n, 1) * 8 + (size_t)J.T.n + 16;
    if (*bytes > 150 * 1024) return fail(ORB_ENOTSUP, "matcher state exceeds LDS (too many keypoints/queries)");
    return ORB_OK;
}

int run_job(const Call& C, const Job& J0) {
    hipStream_t s = C.ctx->stream;
    // the projection-family matchers: the fixed-point resolver where its state fits (it also
    // takes targets k_resolve's per-target LDS state cannot: 8 B per target instead of 13), fed
    // TOPK_FIX-entry candidate lists
    const bool fixMode = J0.outByTarget && (J0.mode == M_LOCAL || (RF_ALL_MODES && (J0.mode == M_WINDOW || J0.mode == M_F2F ||
                                                                                     J0.mode == M_MOTION || J0.mode == M_RELOC ||
                                                                                     J0.mode == M_SIM3P)));
    const bool useFix = fixMode && resolve_fix_lds(J0) <= 150 * 1024;
    Job J = J0;
    // (32 entries: no exact rescan left in the motion-model projection / WindowSearch of the
    // latency probe, 173 / 301 per call with 8; the local-map search has none with 8 and pays
    // ~4 us for the longer merge)
    J.topS = useFix && RF_LONG_LISTS && J0.mode != M_LOCAL ? TOPK_FIX : TOPK;
    if (J.qn > 0) {
        hipLaunchKernelGGL(k_query_prep, dim3((J.qn + 255) / 256), dim3(256), 0, s, J);
        if (J.topS == TOPK_FIX)
            hipLaunchKernelGGL(k_query_scan<TOPK_FIX>, dim3((J.qn + 3) / 4), dim3(256), 0, s, J);
        else
            hipLaunchKernelGGL(k_query_scan<TOPK>, dim3((J.qn + 3) / 4), dim3(256), 0, s, J);
    }
    if (useFix) {
        static std::atomic<bool> fix_attr[64] = {};
        if (!fix_attr[C.device].load()) {
#define SET_FIX_LDS(M) HIPCHK(hipFuncSetAttribute((const void*)k_resolve_fix<M>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024))
            SET_FIX_LDS(M_LOCAL);
            SET_FIX_LDS(M_WINDOW);
            SET_FIX_LDS(M_F2F);
            SET_FIX_LDS(M_MOTION);
            SET_FIX_LDS(M_RELOC);
            SET_FIX_LDS(M_SIM3P);
#undef SET_FIX_LDS
            fix_attr[C.device] = true;
        }
        const size_t fl = resolve_fix_lds(J);
        switch (J.mode) {
#define LAUNCH_FIX(M) \
    case M: hipLaunchKernelGGL(k_resolve_fix<M>, dim3(1), dim3(RF_THREADS), fl, s, J); break;
            LAUNCH_FIX(M_LOCAL)
            LAUNCH_FIX(M_WINDOW)
            LAUNCH_FIX(M_F2F)
            LAUNCH_FIX(M_MOTION)
            LAUNCH_FIX(M_RELOC)
            LAUNCH_FIX(M_SIM3P)
#undef LAUNCH_FIX
            default:
                return fail(ORB_EINVAL, "matcher mode without a fixed-point resolver");
        }
        HIPCHK(hipGetLastError());
        return ORB_OK;
    }
    size_t lds = 0;
    int st = resolve_lds(J, &lds);
    if (st) return st;
    static std::atomic<bool> attr_set[64] = {};
    if (!attr_set[C.device].load()) {
#define SET_RESOLVE_LDS(M) HIPCHK(hipFuncSetAttribute((const void*)k_resolve<M>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024))
        SET_RESOLVE_LDS(M_LOCAL);
        SET_RESOLVE_LDS(M_WINDOW);
        SET_RESOLVE_LDS(M_F2F);
        SET_RESOLVE_LDS(M_MOTION);
        SET_RESOLVE_LDS(M_RELOC);
        SET_RESOLVE_LDS(M_SIM3P);
        SET_RESOLVE_LDS(M_FUSE);
        SET_RESOLVE_LDS(M_FUSE_SCW);
        SET_RESOLVE_LDS(M_SIM3);
        SET_RESOLVE_LDS(M_BOW_KFF);
        SET_RESOLVE_LDS(M_BOW_KFKF);
        SET_RESOLVE_LDS(M_TRIANG);
#undef SET_RESOLVE_LDS
        attr_set[C.device] = true;
    }
    switch (J.mode) {
#define LAUNCH_RESOLVE(M) \
    case M: hipLaunchKernelGGL(k_resolve<M>, dim3(1), dim3(256), lds, s, J); break;
        LAUNCH_RESOLVE(M_LOCAL)
        LAUNCH_RESOLVE(M_WINDOW)
        LAUNCH_RESOLVE(M_F2F)
        LAUNCH_RESOLVE(M_MOTION)
        LAUNCH_RESOLVE(M_RELOC)
        LAUNCH_RESOLVE(M_SIM3P)
        LAUNCH_RESOLVE(M_FUSE)
        LAUNCH_RESOLVE(M_FUSE_SCW)
        LAUNCH_RESOLVE(M_SIM3)
        LAUNCH_RESOLVE(M_BOW_KFF)
        LAUNCH_RESOLVE(M_BOW_KFKF)
        LAUNCH_RESOLVE(M_TRIANG)
#undef LAUNCH_RESOLVE
        default:
            return fail(ORB_EINVAL, "matcher mode without a resolver");
    }
    HIPCHK(hipGetLastError());
    return ORB_OK;
}

Job base_job(int mode) {
    Job J;
    std::memset(&J, 0, sizeof(J));
    J.mode = mode;
    J.nnratio = 0.6f;
    J.th = 1.0f;
    J.thDist = TH_HIGH;
    return J;
}

bool bad_fv(const orb_feature_vector_t& f, int n) {
    if (f.n_nodes < 0) return true;
    if (f.n_nodes == 0) return false;
    if (!f.nodes || !f.offsets || !f.features || f.offsets[0] != 0) return true;
    for (int a = 0; a < f.n_nodes; ++a) {
        if (f.offsets[a + 1] < f.offsets[a]) return true;
        if (a && f.nodes[a] <= f.nodes[a - 1]) return true;
    }
    for (int i = 0; i < f.offsets[f.n_nodes]; ++i)
        if (f.features[i] < 0 || f.features[i] >= n) return true;
    return f.offsets[f.n_nodes] > 65535;
}

// Every feature index at most once in the FeatureVector and no node without features (what
// TemplatedVocabulary::transform builds: FeatureVector::addFeature once per feature).
bool unique_fv(const orb_feature_vector_t& f, int n) {
    std::vector<uint8_t> seen((size_t)std::max(n, 1), 0);
    for (int a = 0; a < f.n_nodes; ++a) {
        if (f.offsets[a + 1] == f.offsets[a]) return false;
        for (int i = f.offsets[a]; i < f.offsets[a + 1]; ++i) {
            if (seen[f.features[i]]) return false;
            seen[f.features[i]] = 1;
        }
    }
    return true;
}

// SearchByBoW (KF-F / KF-KF) of one pair through the batched node-parallel kernel
// (csrc/orb_bow.hip, P = 1): the two frames staged in its [2][cap] layout, one H2D copy, one
// launch, one D2H copy.  (The generic path below replays every query on one wave.)
int bow_match_nodes(int mode, const orb_frame_view_t* V1, const uint8_t* flag1, const orb_feature_vector_t& fv1,
                    const orb_frame_view_t* V2, const uint8_t* flag2, const orb_feature_vector_t& fv2, float nnratio,
                    int check_ori, int32_t* out, int outN, int* n_out, int device) {
    int st;
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    Arena& A = C.A;
    const int cap = std::max(V1->n, V2->n);
    const int counts[2] = {V1->n, V2->n}, fvn[2] = {fv1.n_nodes, fv2.n_nodes}, pair[2] = {0, 1};
    const size_t oK = A.take((size_t)2 * cap * sizeof(orb_keypoint_t));
    A.put(oK, V1->kps, (size_t)V1->n * sizeof(orb_keypoint_t));
    A.put(oK + (size_t)cap * sizeof(orb_keypoint_t), V2->kps, (size_t)V2->n * sizeof(orb_keypoint_t));
    const size_t oD = A.take((size_t)2 * cap * 32);
    A.put(oD, V1->desc, (size_t)V1->n * 32);
    A.put(oD + (size_t)cap * 32, V2->desc, (size_t)V2->n * 32);
    const size_t oC = A.stage(counts, sizeof(counts));
    const size_t oN = A.take((size_t)2 * cap * 4);
    A.put(oN, fv1.nodes, (size_t)fv1.n_nodes * 4);
    A.put(oN + (size_t)cap * 4, fv2.nodes, (size_t)fv2.n_nodes * 4);
    const size_t oO = A.take((size_t)2 * (cap + 1) * 4);
    A.put(oO, fv1.offsets, (size_t)(fv1.n_nodes + 1) * 4);
    A.put(oO + (size_t)(cap + 1) * 4, fv2.offsets, (size_t)(fv2.n_nodes + 1) * 4);
    const size_t oF = A.take((size_t)2 * cap * 4);
    A.put(oF, fv1.features, (size_t)fv1.offsets[fv1.n_nodes] * 4);
    A.put(oF + (size_t)cap * 4, fv2.features, (size_t)fv2.offsets[fv2.n_nodes] * 4);
    const size_t oV = A.stage(fvn, sizeof(fvn));
    const size_t oP = A.stage(pair, sizeof(pair));
    const size_t oU = A.take((size_t)2 * cap);
    A.put(oU, flag1, (size_t)V1->n);
    if (flag2) A.put(oU + (size_t)cap, flag2, (size_t)V2->n);
    const size_t oM = A.take((size_t)cap * 4 + 4);
    if ((st = C.commit())) return st;
    st = orb_search_by_bow_batch_device(mode == M_BOW_KFKF, C.at<orb_keypoint_t>(oK), C.at<uint8_t>(oD), C.at<int32_t>(oC),
                                        cap, C.at<uint32_t>(oN), C.at<int32_t>(oO), C.at<int32_t>(oF), C.at<int32_t>(oV), 1,
                                        C.at<int32_t>(oP), C.at<int32_t>(oP) + 1, C.at<uint8_t>(oU), nnratio, check_ori,
                                        C.at<int32_t>(oM), C.at<int32_t>(oM) + cap, C.ctx->stream);
    if (st) return st;
    int nm = 0;
    if ((st = C.download(out, oM, (size_t)outN * 4)) || (st = C.download(&nm, oM + (size_t)cap * 4, 4)) || (st = C.sync()))
        return st;
    *n_out = nm;
    return ORB_OK;
}

// Shared driver of the three BoW matchers.
int bow_match(int mode, const orb_frame_view_t* V1, const uint8_t* flag1, orb_feature_vector_t fv1,
              const orb_frame_view_t* V2, const uint8_t* flag2, orb_feature_vector_t fv2, const float* F12,
              float nnratio, int check_ori, int32_t* out, int* n_out, int device) {
    int st;
    if ((st = check_view(V1, "query frame")) || (st = check_view(V2, "target frame"))) return st;
    if (!out || !n_out || !flag1 || (mode != M_BOW_KFF && !flag2) || (mode == M_TRIANG && !F12))
        return fail(ORB_EINVAL, "bad arguments");
    if (bad_fv(fv1, V1->n) || bad_fv(fv2, V2->n)) return fail(ORB_EINVAL, "malformed FeatureVector");
    const bool byTarget = mode == M_BOW_KFF;
    const int outN = byTarget ? V2->n : V1->n;
    *n_out = 0;
    if (V1->n == 0 || V2->n == 0 || fv1.n_nodes == 0 || fv2.n_nodes == 0) {
        for (int i = 0; i < outN; ++i) out[i] = -1;
        return ORB_OK;
    }
    if (mode != M_TRIANG && std::max(V1->n, V2->n) <= 8192 && fv1.n_nodes <= V1->n && fv2.n_nodes <= V2->n &&
        unique_fv(fv1, V1->n) && unique_fv(fv2, V2->n))
        return bow_match_nodes(mode, V1, flag1, fv1, V2, flag2, fv2, nnratio, check_ori, out, outN, n_out, device);
    const int qn = fv1.offsets[fv1.n_nodes];
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    Arena& A = C.A;
    const size_t o1k = A.stage(V1->kps, (size_t)V1->n * sizeof(orb_keypoint_t));
    const size_t o1d = A.stage(V1->desc, (size_t)V1->n * 32);
    const size_t o1f = A.stage(flag1, (size_t)V1->n);
    const size_t o2k = A.stage(V2->kps, (size_t)V2->n * sizeof(orb_keypoint_t));
    const size_t o2d = A.stage(V2->desc, (size_t)V2->n * 32);
    const size_t o2f = flag2 ? A.stage(flag2, (size_t)V2->n) : 0;
    const size_t on1 = A.stage(fv1.nodes, (size_t)fv1.n_nodes * 4);
    const size_t oo1 = A.stage(fv1.offsets, (size_t)(fv1.n_nodes + 1) * 4);
    const size_t of1 = A.stage(fv1.features, (size_t)qn * 4);
    const size_t on2 = A.stage(fv2.nodes, (size_t)fv2.n_nodes * 4);
    const size_t oo2 = A.stage(fv2.offsets, (size_t)(fv2.n_nodes + 1) * 4);
    const size_t of2 = A.stage(fv2.features, (size_t)fv2.offsets[fv2.n_nodes] * 4);
    const JobOffs jo = plan_job(A, qn, outN);
    if ((st = C.commit())) return st;
    Job J = base_job(mode);
    J.T.kps = C.at<orb_keypoint_t>(o2k);
    J.T.desc = C.at<uint32_t>(o2d);
    J.T.n = V2->n;
    J.T.nlevels = V2->nlevels;
    std::memcpy(J.T.sigma2, V2->level_sigma2, sizeof(J.T.sigma2));
    std::memcpy(J.T.sf, V2->scale_factors, sizeof(J.T.sf));
    J.T.items = C.at<int>(of2);
    J.qkps = C.at<orb_keypoint_t>(o1k);
    J.qdesc = C.at<uint32_t>(o1d);
    J.qflag = C.at<uint8_t>(o1f);
    J.tflag = flag2 ? C.at<uint8_t>(o2f) : nullptr;
    J.fv1Nodes = C.at<uint32_t>(on1);
    J.fv1Off = C.at<int>(oo1);
    J.fv1Feat = C.at<int>(of1);
    J.fv1N = fv1.n_nodes;
    J.fv2Nodes = C.at<uint32_t>(on2);
    J.fv2Off = C.at<int>(oo2);
    J.fv2N = fv2.n_nodes;
    J.nnratio = nnratio;
    J.checkOri = check_ori;
    if (F12) std::memcpy(J.F12, F12, sizeof(J.F12));
    J.outByTarget = byTarget;
    bind_job(C, J, jo, qn, outN);
    if ((st = run_job(C, J))) return st;
    int nm = 0;
    if ((st = C.download(out, jo.out, (size_t)outN * 4)) || (st = C.download(&nm, jo.nOut, 4)) || (st = C.sync()))
        return st;
    *n_out = nm;
    return ORB_OK;
}

// Shared driver of the grid matchers: target view + queries -> one job.
struct GridQueries {
    int qn = 0;
    const uint8_t* flag = nullptr;
    const uint8_t* desc = nullptr;        // qn x 32 (or the query frame's descriptors)
    const orb_keypoint_t* kps = nullptr;  // query frame keypoints (qn)
    const float* pos = nullptr;
    const float* normal = nullptr;
    const float* dmin = nullptr;
    const float* dmax = nullptr;
    const float* u = nullptr;
    const float* v = nullptr;
    const int32_t* level = nullptr;
    int levelStride = 1;
    const float* vcos = nullptr;
};

int grid_match(Job J, const orb_frame_view_t* T, const uint8_t* taken, const GridQueries& Q, int32_t* out,
               int* n_out, int device, int outByTarget) {
    int st;
    if ((st = check_view(T, "target frame"))) return st;
    if (!out || !n_out || Q.qn < 0) return fail(ORB_EINVAL, "bad arguments");
    const int outN = outByTarget ? T->n : Q.qn;
    *n_out = 0;
    if (T->n == 0 || Q.qn == 0) {
        for (int i = 0; i < outN; ++i) out[i] = -1;
        return ORB_OK;
    }
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    Arena& A = C.A;
    const ViewOffs vo = plan_view(A, T, true);
    const size_t oTaken = taken ? A.stage(taken, (size_t)T->n) : 0;
    const size_t oFlag = Q.flag ? A.stage(Q.flag, (size_t)Q.qn) : 0;
    const size_t oDesc = Q.desc ? A.stage(Q.desc, (size_t)Q.qn * 32) : 0;
    const size_t oKps = Q.kps ? A.stage(Q.kps, (size_t)Q.qn * sizeof(orb_keypoint_t)) : 0;
    const size_t oPos = Q.pos ? A.stage(Q.pos, (size_t)Q.qn * 12) : 0;
    const size_t oNrm = Q.normal ? A.stage(Q.normal, (size_t)Q.qn * 12) : 0;
    const size_t oDmin = Q.dmin ? A.stage(Q.dmin, (size_t)Q.qn * 4) : 0;
    const size_t oDmax = Q.dmax ? A.stage(Q.dmax, (size_t)Q.qn * 4) : 0;
    const size_t oU = Q.u ? A.stage(Q.u, (size_t)Q.qn * 4) : 0;
    const size_t oV = Q.v ? A.stage(Q.v, (size_t)Q.qn * 4) : 0;
    const size_t oL = Q.level ? A.stage(Q.level, (size_t)Q.qn * 4 * Q.levelStride) : 0;
    const size_t oC = Q.vcos ? A.stage(Q.vcos, (size_t)Q.qn * 4) : 0;
    const JobOffs jo = plan_job(A, Q.qn, outN);
    if ((st = C.commit())) return st;
    J.T = make_dview(C, T, vo, true);
    if ((st = launch_grid(C, J.T))) return st;
    J.taken0 = taken ? C.at<uint8_t>(oTaken) : nullptr;
    J.qflag = Q.flag ? C.at<uint8_t>(oFlag) : nullptr;
    J.qdesc = Q.desc ? C.at<uint32_t>(oDesc) : nullptr;
    J.qkps = Q.kps ? C.at<orb_keypoint_t>(oKps) : nullptr;
    J.qpos = Q.pos ? C.at<float>(oPos) : nullptr;
    J.qnormal = Q.normal ? C.at<float>(oNrm) : nullptr;
    J.qdmin = Q.dmin ? C.at<float>(oDmin) : nullptr;
    J.qdmax = Q.dmax ? C.at<float>(oDmax) : nullptr;
    J.qu = Q.u ? C.at<float>(oU) : nullptr;
    J.qv = Q.v ? C.at<float>(oV) : nullptr;
    J.qlevel = Q.level ? C.at<int>(oL) : nullptr;
    J.qvcos = Q.vcos ? C.at<float>(oC) : nullptr;
    J.outByTarget = outByTarget;
    bind_job(C, J, jo, Q.qn, outN);
    if ((st = run_job(C, J))) return st;
    int nm = 0;
    if ((st = C.download(out, jo.out, (size_t)outN * 4)) || (st = C.download(&nm, jo.nOut, 4)) || (st = C.sync()))
        return st;
    if (nm < 0) return fail(ORB_EDEVICE, "local-map resolver did not converge");
    *n_out = nm;
    return ORB_OK;
}

bool finite_pose(const orb_frame_view_t* v) {
    for (int i = 0; i < 9; ++i)
        if (!std::isfinite(v->Rcw[i])) return false;
    for (int i = 0; i < 3; ++i)
        if (!std::isfinite(v->tcw[i]) || !std::isfinite(v->Ow[i])) return false;
    return true;
}

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
extern "C" {

int orb_features_in_area(const orb_frame_view_t* view, int keyframe, int q, const float* x, const float* y,
                         const float* r, const int32_t* min_level, const int32_t* max_level, int32_t* out_offsets,
                         int32_t* out_indices, int capacity, int device) {
    int st;
    if ((st = check_view(view, "frame"))) return st;
    if (q < 0 || !out_offsets || (q > 0 && (!x || !y || !r)) || capacity < 0 || (capacity > 0 && !out_indices))
        return fail(ORB_EINVAL, "bad arguments");
    if (!keyframe && ((min_level == nullptr) != (max_level == nullptr)))
        return fail(ORB_EINVAL, "min_level and max_level go together");
    out_offsets[0] = 0;
    if (q == 0) return ORB_OK;
    if (view->n == 0) {
        for (int i = 0; i <= q; ++i) out_offsets[i] = 0;
        return ORB_OK;
    }
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    Arena& A = C.A;
    const ViewOffs vo = plan_view(A, view, true);
    const size_t ox = A.stage(x, (size_t)q * 4), oy = A.stage(y, (size_t)q * 4), orr = A.stage(r, (size_t)q * 4);
    std::vector<int32_t> lv;
    size_t ol = 0;
    if (!keyframe && min_level) {
        lv.resize((size_t)2 * q);
        for (int i = 0; i < q; ++i) {
            lv[2 * i] = min_level[i];
            lv[2 * i + 1] = max_level[i];
        }
        ol = A.stage(lv.data(), lv.size() * 4);
    }
    const JobOffs jo = plan_job(A, q, 1);
    const size_t oOff = A.take((size_t)(q + 1) * 4);
    const size_t oOut = A.take((size_t)std::max(capacity, 1) * 4);
    if ((st = C.commit())) return st;
    Job J = base_job(keyframe ? M_AREA_KF : M_AREA_F);
    J.T = make_dview(C, view, vo, true);
    if ((st = launch_grid(C, J.T))) return st;
    J.qu = C.at<float>(ox);
    J.qv = C.at<float>(oy);
    J.qvcos = C.at<float>(orr);
    J.qlevel = ol ? C.at<int>(ol) : nullptr;
    bind_job(C, J, jo, q, 1);
    J.areaOff = C.at<int>(oOff);
    J.areaOut = C.at<int>(oOut);
    hipStream_t s = C.ctx->stream;
    hipLaunchKernelGGL(k_query_prep, dim3((q + 255) / 256), dim3(256), 0, s, J);
    hipLaunchKernelGGL(k_query_scan<TOPK>, dim3((q + 3) / 4), dim3(256), 0, s, J);
    HIPCHK(hipGetLastError());
    std::vector<int> cnt(q);
    if ((st = C.download(cnt.data(), jo.cnt, (size_t)q * 4)) || (st = C.sync())) return st;
    long long tot = 0;
    for (int i = 0; i < q; ++i) {
        out_offsets[i] = (int32_t)std::min<long long>(tot, INT_MAX);
        tot += cnt[i];
    }
    out_offsets[q] = (int32_t)std::min<long long>(tot, INT_MAX);
    if (tot > capacity) return fail(ORB_ERANGE, "candidate capacity too small");
    if (tot == 0) return ORB_OK;
    HIPCHK(hipMemcpyAsync(J.areaOff, out_offsets, (size_t)(q + 1) * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_area_fill, dim3((q + 3) / 4), dim3(256), 0, s, J);
    HIPCHK(hipGetLastError());
    if ((st = C.download(out_indices, oOut, (size_t)tot * 4)) || (st = C.sync())) return st;
    return ORB_OK;
}

int orb_frame_is_in_frustum(const orb_frame_view_t* F, orb_map_points_t mps, float viewing_cos_limit,
                            uint8_t* in_view, float* proj_x, float* proj_y, int32_t* level, float* view_cos,
                            int device);

int orb_search_by_bow_kf_f(const orb_frame_view_t* KF, const uint8_t* kf_usable, orb_feature_vector_t kf_fv,
                           const orb_frame_view_t* F, orb_feature_vector_t f_fv, float nnratio, int check_ori,
                           int32_t* f_match, int* n_matches, int device) {
    return bow_match(M_BOW_KFF, KF, kf_usable, kf_fv, F, nullptr, f_fv, nullptr, nnratio, check_ori, f_match,
                     n_matches, device);
}

int orb_search_by_bow_kf_kf(const orb_frame_view_t* KF1, const uint8_t* usable1, orb_feature_vector_t fv1,
                            const orb_frame_view_t* KF2, const uint8_t* usable2, orb_feature_vector_t fv2,
                            float nnratio, int check_ori, int32_t* match12, int* n_matches, int device) {
    return bow_match(M_BOW_KFKF, KF1, usable1, fv1, KF2, usable2, fv2, nullptr, nnratio, check_ori, match12,
                     n_matches, device);
}

int orb_search_for_triangulation(const orb_frame_view_t* KF1, const uint8_t* has_mp1, orb_feature_vector_t fv1,
                                 const orb_frame_view_t* KF2, const uint8_t* has_mp2, orb_feature_vector_t fv2,
                                 const float* F12, float nnratio, int check_ori, int32_t* match12, int* n_matches,
                                 int device) {
    return bow_match(M_TRIANG, KF1, has_mp1, fv1, KF2, has_mp2, fv2, F12, nnratio, check_ori, match12, n_matches,
                     device);
}

int orb_window_search(const orb_frame_view_t* F1, const uint8_t* usable1, const orb_frame_view_t* F2, int window,
                      int min_scale_level, int max_scale_level, float nnratio, int check_ori, int32_t* match21,
                      int* n_matches, int device) {
    int st;
    if ((st = check_view(F1, "F1"))) return st;
    if (F1->n && !usable1) return fail(ORB_EINVAL, "usable1 is NULL");
    Job J = base_job(M_WINDOW);
    J.window = window;
    J.minLevel = min_scale_level;
    J.maxLevel = max_scale_level;
    J.nnratio = nnratio;
    J.checkOri = check_ori;
    GridQueries Q;
    Q.qn = F1->n;
    Q.flag = usable1;
    Q.desc = F1->desc;
    Q.kps = F1->kps;
    return grid_match(J, F2, nullptr, Q, match21, n_matches, device, 1);
}

int orb_search_by_projection_local(const orb_frame_view_t* F, const uint8_t* f_taken, int n_mp, const uint8_t* usable,
                                   const float* proj_x, const float* proj_y, const int32_t* level,
                                   const float* view_cos, const uint8_t* mp_desc, float th, float nnratio,
                                   int32_t* f_match, int* n_matches, int device) {
    int st;
    if ((st = check_view(F, "F"))) return st;
    if (n_mp < 0 || (n_mp > 0 && (!usable || !proj_x || !proj_y || !level || !view_cos || !mp_desc)))
        return fail(ORB_EINVAL, "bad MapPoint arrays");
    for (int i = 0; i < n_mp; ++i)
        if (usable[i] && (level[i] < 0 || level[i] >= F->nlevels)) return fail(ORB_EINVAL, "predicted level out of range");
    Job J = base_job(M_LOCAL);
    J.th = th;
    J.nnratio = nnratio;
    GridQueries Q;
    Q.qn = n_mp;
    Q.flag = usable;
    Q.desc = mp_desc;
    Q.u = proj_x;
    Q.v = proj_y;
    Q.level = level;
    Q.vcos = view_cos;
    return grid_match(J, F, f_taken, Q, f_match, n_matches, device, 1);
}

int orb_search_by_projection_f2f(const orb_frame_view_t* F1, orb_map_points_t mp1, const uint8_t* usable1,
                                 const orb_frame_view_t* F2, const uint8_t* f2_taken, int window, float nnratio,
                                 int32_t* match2, int* n_matches, int device) {
    int st;
    if ((st = check_view(F1, "F1"))) return st;
    if (F1->n && (!usable1 || !mp1.pos || mp1.n < F1->n)) return fail(ORB_EINVAL, "bad F1 MapPoint arrays");
    if (!finite_pose(F2)) return fail(ORB_EINVAL, "F2 pose not finite");
    Job J = base_job(M_F2F);
    J.window = window;
    J.nnratio = nnratio;
    GridQueries Q;
    Q.qn = F1->n;
    Q.flag = usable1;
    Q.desc = F1->desc;
    Q.kps = F1->kps;
    Q.pos = mp1.pos;
    return grid_match(J, F2, f2_taken, Q, match2, n_matches, device, 1);
}

int orb_search_by_projection_motion(const orb_frame_view_t* Cur, const uint8_t* cur_taken, const orb_frame_view_t* Last,
                                    orb_map_points_t mp, const uint8_t* usable, float th, int check_ori,
                                    int32_t* cur_match, int* n_matches, int device) {
    int st;
    if ((st = check_view(Last, "LastFrame"))) return st;
    if (Last->n && (!usable || !mp.pos || mp.n < Last->n)) return fail(ORB_EINVAL, "bad LastFrame MapPoint arrays");
    if (Cur && Last->nlevels > Cur->nlevels) return fail(ORB_EINVAL, "LastFrame has more levels than CurrentFrame");
    Job J = base_job(M_MOTION);
    J.th = th;
    J.checkOri = check_ori;
    GridQueries Q;
    Q.qn = Last->n;
    Q.flag = usable;
    Q.desc = Last->desc;
    Q.kps = Last->kps;
    Q.pos = mp.pos;
    return grid_match(J, Cur, cur_taken, Q, cur_match, n_matches, device, 1);
}

int orb_search_by_projection_reloc(const orb_frame_view_t* Cur, const uint8_t* cur_taken, const orb_frame_view_t* KF,
                                   orb_map_points_t mp, const uint8_t* usable, float th, int orb_dist,
                                   int check_ori, int32_t* cur_match, int* n_matches, int device) {
    int st;
    if ((st = check_view(KF, "KF"))) return st;
    if (KF->n && (!usable || !mp.pos || !mp.dmin || !mp.desc || mp.n < KF->n))
        return fail(ORB_EINVAL, "bad KF MapPoint arrays");
    Job J = base_job(M_RELOC);
    J.th = th;
    J.thDist = orb_dist;
    J.checkOri = check_ori;
    GridQueries Q;
    Q.qn = KF->n;
    Q.flag = usable;
    Q.desc = mp.desc;
    Q.kps = KF->kps;
    Q.pos = mp.pos;
    Q.dmin = mp.dmin;
    return grid_match(J, Cur, cur_taken, Q, cur_match, n_matches, device, 1);
}

int orb_search_by_projection_sim3(const orb_frame_view_t* KF, const uint8_t* kf_taken, orb_map_points_t pts,
                                  const uint8_t* usable, int th, int32_t* kf_match, int* n_matches, int device) {
    if (pts.n < 0 || (pts.n > 0 && (!usable || !pts.pos || !pts.normal || !pts.dmin || !pts.dmax || !pts.desc)))
        return fail(ORB_EINVAL, "bad point arrays");
    Job J = base_job(M_SIM3P);
    J.th = (float)th;
    J.thDist = TH_LOW;
    GridQueries Q;
    Q.qn = pts.n;
    Q.flag = usable;
    Q.desc = pts.desc;
    Q.pos = pts.pos;
    Q.normal = pts.normal;
    Q.dmin = pts.dmin;
    Q.dmax = pts.dmax;
    return grid_match(J, KF, kf_taken, Q, kf_match, n_matches, device, 1);
}

int orb_fuse(const orb_frame_view_t* KF, orb_map_points_t pts, const uint8_t* usable, float th, int scw,
             int32_t* best_idx, int* n_fused, int device) {
    if (pts.n < 0 || (pts.n > 0 && (!usable || !pts.pos || !pts.normal || !pts.dmin || !pts.dmax || !pts.desc)))
        return fail(ORB_EINVAL, "bad point arrays");
    Job J = base_job(scw ? M_FUSE_SCW : M_FUSE);
    J.th = th;
    J.thDist = TH_LOW;
    GridQueries Q;
    Q.qn = pts.n;
    Q.flag = usable;
    Q.desc = pts.desc;
    Q.pos = pts.pos;
    Q.normal = pts.normal;
    Q.dmin = pts.dmin;
    Q.dmax = pts.dmax;
    return grid_match(J, KF, nullptr, Q, best_idx, n_fused, device, 0);
}

int orb_search_by_sim3(const orb_frame_view_t* KF1, orb_map_points_t mp1, const uint8_t* usable1,
                       const orb_frame_view_t* KF2, orb_map_points_t mp2, const uint8_t* usable2, const float* sR12,
                       const float* t12, const float* sR21, const float* t21, float th, int32_t* match12,
                       int* n_found, int device) {
    int st;
    if ((st = check_view(KF1, "KF1")) || (st = check_view(KF2, "KF2"))) return st;
    if (!sR12 || !t12 || !sR21 || !t21 || !match12 || !n_found) return fail(ORB_EINVAL, "bad arguments");
    if ((KF1->n && (!usable1 || !mp1.pos || !mp1.dmin || !mp1.dmax || !mp1.desc || mp1.n < KF1->n)) ||
        (KF2->n && (!usable2 || !mp2.pos || !mp2.dmin || !mp2.dmax || !mp2.desc || mp2.n < KF2->n)))
        return fail(ORB_EINVAL, "bad MapPoint arrays");
    // direction 1: KF1's points into KF2 -> vnMatch1 (n1); direction 2: KF2's into KF1 -> vnMatch2 (n2)
    std::vector<int32_t> m1(KF1->n), m2(KF2->n);
    int n1 = 0, n2 = 0;
    for (int dir = 0; dir < 2; ++dir) {
        const orb_frame_view_t* src = dir ? KF2 : KF1;
        const orb_frame_view_t* dst = dir ? KF1 : KF2;
        const orb_map_points_t& mp = dir ? mp2 : mp1;
        Job J = base_job(M_SIM3);
        J.th = th;
        J.thDist = TH_HIGH;
        std::memcpy(J.SRw, src->Rcw, sizeof(J.SRw));
        std::memcpy(J.Stw, src->tcw, sizeof(J.Stw));
        std::memcpy(J.SR, dir ? sR12 : sR21, sizeof(J.SR));
        std::memcpy(J.St, dir ? t12 : t21, sizeof(J.St));
        J.qfx = KF1->fx;  // pKF1's calibration for both directions (ORBmatcher.cc:1270-1273)
        J.qfy = KF1->fy;
        J.qcx = KF1->cx;
        J.qcy = KF1->cy;
        GridQueries Q;
        Q.qn = src->n;
        Q.flag = dir ? usable2 : usable1;
        Q.desc = mp.desc;
        Q.pos = mp.pos;
        Q.dmin = mp.dmin;
        Q.dmax = mp.dmax;
        if ((st = grid_match(J, dst, nullptr, Q, dir ? m2.data() : m1.data(), dir ? &n2 : &n1, device, 0))) return st;
    }
    // agreement on the device of the call (tiny; keeps the selection off the host)
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    const size_t o1 = C.A.stage(m1.data(), m1.size() * 4), o2 = C.A.stage(m2.data(), m2.size() * 4);
    const size_t oo = C.A.take(std::max<size_t>(m1.size(), 1) * 4), on = C.A.take(16);
    if ((st = C.commit())) return st;
    hipLaunchKernelGGL(k_sim3_agree, dim3(1), dim3(256), 0, C.ctx->stream, C.at<int>(o1), KF1->n, C.at<int>(o2),
                       C.at<int>(oo), C.at<int>(on));
    HIPCHK(hipGetLastError());
    int nf = 0;
    if ((st = C.download(match12, oo, m1.size() * 4)) || (st = C.download(&nf, on, 4)) || (st = C.sync())) return st;
    *n_found = nf;
    return ORB_OK;
}

}  // extern "C"

// ---- Frame::isInFrustum (Frame.cc:137-198), one thread per MapPoint ----------------------
namespace {
__global__ void __launch_bounds__(256) k_is_in_frustum(DView T, const float* __restrict__ pos,
                                                       const float* __restrict__ normal, const float* __restrict__ dmin,
                                                       const float* __restrict__ dmax, int n, float limit,
                                                       uint8_t* __restrict__ inView, float* __restrict__ px,
                                                       float* __restrict__ py, int* __restrict__ lv,
                                                       float* __restrict__ vc) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t ok = 0;
    float u = 0.f, v = 0.f, viewCos = 0.f;
    int pred = -1;
    do {
        const float* P = pos + 3 * i;
        float Pc[3];
        gemm3_add(T.R, P, T.t, Pc);
        const float PcX = Pc[0], PcY = Pc[1], PcZ = Pc[2];
        if (PcZ < 0.0f) break;
        const float invz = (float)(1.0 / (double)PcZ);
        const float uu = __builtin_fmaf(T.fx * PcX, invz, T.cx);
        const float vv = __builtin_fmaf(T.fy * PcY, invz, T.cy);
        if (uu < (float)T.minX || uu > (float)T.maxX) break;
        if (vv < (float)T.minY || vv > (float)T.maxY) break;
        const float maxDistance = dmax[i], minDistance = dmin[i];
        float PO[3] = {P[0] - T.Ow[0], P[1] - T.Ow[1], P[2] - T.Ow[2]};
        const float dist = (float)norm3(PO);
        if (dist < minDistance || dist > maxDistance) break;
        const float vcos = (float)(dot3(PO, normal + 3 * i) / (double)dist);
        if (vcos < limit) break;
        const float ratio = dist / minDistance;
        int nPred = 0;
        while (nPred < T.nlevels && T.sf[nPred] < ratio) ++nPred;
        if (nPred >= T.nlevels) nPred = T.nlevels - 1;
        ok = 1;
        u = uu;
        v = vv;
        viewCos = vcos;
        pred = nPred;
    } while (0);
    inView[i] = ok;
    px[i] = u;
    py[i] = v;
    lv[i] = pred;
    vc[i] = viewCos;
}
}  // namespace

extern "C" int orb_frame_is_in_frustum(const orb_frame_view_t* F, orb_map_points_t mps, float viewing_cos_limit,
                                       uint8_t* in_view, float* proj_x, float* proj_y, int32_t* level,
                                       float* view_cos, int device) {
    if (!F || F->nlevels < 1 || F->nlevels > ORB_MAX_VIEW_LEVELS || mps.n < 0 ||
        (mps.n > 0 && (!mps.pos || !mps.normal || !mps.dmin || !mps.dmax || !in_view || !proj_x || !proj_y || !level ||
                       !view_cos)))
        return fail(ORB_EINVAL, "bad arguments");
    if (mps.n == 0) return ORB_OK;
    int st;
    Call C{device};
    if ((st = C.begin())) return st;
    DeviceGuard dg(device);
    Arena& A = C.A;
    const size_t n = (size_t)mps.n;
    const size_t op = A.stage(mps.pos, n * 12), onr = A.stage(mps.normal, n * 12), omn = A.stage(mps.dmin, n * 4),
                 omx = A.stage(mps.dmax, n * 4);
    const size_t oi = A.take(n), ox = A.take(n * 4), oy = A.take(n * 4), ol = A.take(n * 4), oc = A.take(n * 4);
    if ((st = C.commit())) return st;
    orb_frame_view_t Fv = *F;
    Fv.n = 0;
    Fv.kps = nullptr;
    Fv.desc = nullptr;
    ViewOffs vo{};
    DView d = make_dview(C, &Fv, vo, false);
    hipLaunchKernelGGL(k_is_in_frustum, dim3((mps.n + 255) / 256), dim3(256), 0, C.ctx->stream, d, C.at<float>(op),
                       C.at<float>(onr), C.at<float>(omn), C.at<float>(omx), mps.n, viewing_cos_limit,
                       C.at<uint8_t>(oi), C.at<float>(ox), C.at<float>(oy), C.at<int>(ol), C.at<float>(oc));
    HIPCHK(hipGetLastError());
    if ((st = C.download(in_view, oi, n)) || (st = C.download(proj_x, ox, n * 4)) ||
        (st = C.download(proj_y, oy, n * 4)) || (st = C.download(level, ol, n * 4)) ||
        (st = C.download(view_cos, oc, n * 4)) || (st = C.sync()))
        return st;
    return ORB_OK;
}
