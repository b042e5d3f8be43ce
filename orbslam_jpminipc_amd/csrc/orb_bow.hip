// orb_bow.hip — MI355X (gfx950) batched SearchByBoW: many (KeyFrame, Frame) or (KeyFrame,
// KeyFrame) pairs per launch over device-resident extractor output and the FeatureVectors
// orb_vocabulary_transform_batch_device writes (the reference's per-frame
// Frame::ComputeBoW -> ORBmatcher::SearchByBoW chain, Tracking.cc:927 / LoopClosing.cc:278).
//
// Reference loop (ORBmatcher.cc:155-284, 715-850): walk the two FeatureVectors' common vocabulary
// nodes in ascending id order; inside a node, every usable KF feature (in FeatureVector order)
// takes the Hamming best / second best of the node's other-side features not yet matched in this
// call, is accepted by TH_LOW and the ratio test, and marks its target matched; then the three
// dominant rotation-histogram bins are kept.  A target feature sits in exactly ONE node of its
// FeatureVector, so the "already matched" state of a node is touched only by that node's own
// queries: nodes are independent and run in parallel (one wave per node), the queries of a node
// in the reference's order.  Only the rotation filter is per pair.
//
// One 1024-thread workgroup per pair (16 waves: 4 waves per pair left 2 waves per SIMD at 511
// pairs, 0.388 ms per c3 step):
//   0. (where both frames fit, cap <= ~1800) their descriptors, feature lists, node offsets and
//      B's node ids are copied into LDS by all threads, so the node loop below touches LDS only;
//   1. each thread binary-searches KF node positions in the other vector's node list;
//   2. wave w takes the common nodes w, w+16, ...: per query (wave-uniform) every lane scores the
//      node's candidates it holds (<= 64 candidates: one per lane, descriptor and matched flag
//      in registers for the whole node; more: strided, reloaded, flags in LDS), key =
//      (distance << 16) | candidate position, and two wave-min reductions give the reference's
//      bestDist1 / bestIdx (first minimum in candidate order) and bestDist2; an accepted query
//      marks its target and writes the output;
//   3. the rotation histogram from the outputs, ComputeThreeMaxima (ORBmatcher.cc:1748-1789) and
//      the removal pass (bins recomputed from the keypoint angles of the kept outputs).
// Latency-bound by design (sequential queries per node); SURVEY §8d-style bytes per pair:
// 32 B per feature of both frames + 4 B per output slot.
#include <hip/hip_runtime.h>

#include <climits>
#include <mutex>
#include <string>

#include "../../include/orb_abi.h"
#include "orb_device.h"
#include "orb_internal.h"

namespace {

constexpr int TH_LOW = 50, HISTO = 30;  // ORBmatcher.cc:40-42
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int BOW_WAVES = 16;  // waves per pair: the common nodes are dealt round-robin to them
constexpr int BOW_T = 64 * BOW_WAVES;

__device__ __forceinline__ uint32_t wmin(uint32_t v) { return orbdev::wave_min_u32(v); }
// minimum over each 16-lane DPP row, in every lane of the row (row_ror 1, 2, 4, 8)
__device__ __forceinline__ uint32_t rmin16(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x121, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x122, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x124, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false));
    return v;
}
#ifndef BOW_BATCH4
#define BOW_BATCH4 1  // nodes of <= 16 candidates: four queries per step (speculated, exact); 0: one per step
#endif

__device__ __forceinline__ int rot_bin(float a1, float a2) {  // ORBmatcher.cc:230-236 / 799-805
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / HISTO));
    if (bin == HISTO) bin = 0;
    return bin;
}

__device__ __forceinline__ int ham(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

struct BowBatch {
    const orb_keypoint_t* kps;  // [B][cap]
    const uint8_t* desc;        // [B][cap][32]
    const int32_t* counts;      // [B]
    const uint32_t* fvNodes;    // [B][cap]
    const int32_t* fvOff;       // [B][cap + 1]
    const int32_t* fvFeat;      // [B][cap]
    const int32_t* fvN;         // [B]
    const int32_t* pairA;       // [P] KF (KF1) frame
    const int32_t* pairB;       // [P] F (KF2) frame
    const uint8_t* usable;      // [B][cap] or NULL (every feature has a usable MapPoint)
    int32_t* match;             // [P][cap]
    int32_t* nmatches;          // [P]
    int cap, kfkf, checkOri;
    float nnratio;
};

// LDS bytes of the staged variant: both frames' descriptors, feature-vector feature lists and
// node offsets, the usable flags of A and B's node ids, on top of the per-pair state (5 cap)
__host__ __device__ inline size_t bow_stage_bytes(int cap) {
    return ((5 * (size_t)cap + 15) & ~(size_t)15) + 64 * (size_t)cap + 8 * (size_t)cap + 8 * ((size_t)cap + 1) +
           (((size_t)cap + 3) & ~(size_t)3) + 4 * (size_t)cap;
}

// STAGE: both frames' descriptors, feature lists and node offsets are copied into LDS first (all
// threads, coalesced), so a node's queries run on LDS only; without it every node pays ~5
// dependent global round trips (offsets, candidate indices -> descriptors, query indices ->
// flags / descriptors) on its wave.
template <bool STAGE>
__global__ void __launch_bounds__(BOW_T) k_bow_pairs(BowBatch J) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_hist[HISTO];
    __shared__ int s_ind[3];
    __shared__ int s_acc, s_rem;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cap = J.cap;
    const int fa = J.pairA[p], fb = J.pairB[p];
    const int nA = min(J.counts[fa], cap), nB = min(J.counts[fb], cap);
    const int nodesA = min(J.fvN[fa], nA), nodesB = min(J.fvN[fb], nB);
    const uint32_t* NA = J.fvNodes + (size_t)fa * cap;
    const uint32_t* NB = J.fvNodes + (size_t)fb * cap;
    const int32_t* gOA = J.fvOff + (size_t)fa * (cap + 1);
    const int32_t* gOB = J.fvOff + (size_t)fb * (cap + 1);
    const int32_t* gFA = J.fvFeat + (size_t)fa * cap;
    const int32_t* gFB = J.fvFeat + (size_t)fb * cap;
    const orb_keypoint_t* KA = J.kps + (size_t)fa * cap;
    const orb_keypoint_t* KB = J.kps + (size_t)fb * cap;
    const uint4* gDA = (const uint4*)(J.desc + (size_t)fa * cap * 32);
    const uint4* gDB = (const uint4*)(J.desc + (size_t)fb * cap * 32);
    const uint8_t* gUA = J.usable ? J.usable + (size_t)fa * cap : nullptr;
    const uint8_t* UB = J.usable ? J.usable + (size_t)fb * cap : nullptr;
    int32_t* out = J.match + (size_t)p * cap;
    const int nOut = J.kfkf ? nA : nB;  // vpMatches12 over KF1 / vpMapPointMatches over F
    int* s_mb = (int*)smem;                   // [cap] KF node position -> other node position or -1
    uint8_t* s_taken = smem + 4 * (size_t)cap;  // [cap] other-side features matched (or unusable)
    // the staged copies (STAGE), after the per-pair state
    uint4* sDA = (uint4*)(smem + ((5 * (size_t)cap + 15) & ~(size_t)15));
    uint4* sDB = sDA + 2 * (size_t)cap;
    int* sFA = (int*)(sDB + 2 * (size_t)cap);
    int* sFB = sFA + cap;
    int* sOA = sFB + cap;
    int* sOB = sOA + cap + 1;
    uint8_t* sUA = (uint8_t*)(sOB + cap + 1);
    uint32_t* sNB = (uint32_t*)(sUA + ((cap + 3) & ~3));
    const uint4* DA = STAGE ? sDA : gDA;
    const uint4* DB = STAGE ? sDB : gDB;
    const int32_t* FA = STAGE ? sFA : gFA;
    const int32_t* FB = STAGE ? sFB : gFB;
    const int32_t* OA = STAGE ? sOA : gOA;
    const int32_t* OB = STAGE ? sOB : gOB;
    const uint8_t* UA = STAGE ? (gUA ? sUA : nullptr) : gUA;

    for (int i = tid; i < cap; i += BOW_T) out[i] = -1;
    for (int i = tid; i < nB; i += BOW_T) s_taken[i] = (J.kfkf && UB) ? (uint8_t)(UB[i] == 0) : (uint8_t)0;
    if constexpr (STAGE) {
        for (int i = tid; i < 2 * nA; i += BOW_T) sDA[i] = gDA[i];
        for (int i = tid; i < 2 * nB; i += BOW_T) sDB[i] = gDB[i];
        for (int i = tid; i <= nodesA; i += BOW_T) sOA[i] = gOA[i];
        for (int i = tid; i <= nodesB; i += BOW_T) sOB[i] = gOB[i];
        for (int i = tid; i < nA; i += BOW_T) sFA[i] = gFA[i];  // (a vector's features: at most its frame's)
        for (int i = tid; i < nB; i += BOW_T) sFB[i] = gFB[i];
        if (gUA)
            for (int i = tid; i < nA; i += BOW_T) sUA[i] = gUA[i];
        for (int i = tid; i < nodesB; i += BOW_T) sNB[i] = NB[i];
        __syncthreads();  // the lower_bound below searches B's node ids in LDS
    }
    const uint32_t* NBs = STAGE ? sNB : NB;
    for (int a = tid; a < nodesA; a += BOW_T) {  // the merge walk's common nodes (lower_bound)
        const uint32_t id = NA[a];
        int lo = 0, hi = nodesB;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (NBs[mid] < id)
                lo = mid + 1;
            else
                hi = mid;
        }
        s_mb[a] = (lo < nodesB && NBs[lo] == id) ? lo : -1;
    }
    if (tid < HISTO) s_hist[tid] = 0;
    if (tid == 0) s_acc = 0, s_rem = 0;
    __syncthreads();

    int acc = 0;  // accepted by this wave (lane 0 counts)
    for (int a = wave; a < nodesA; a += BOW_WAVES) {
        const int b = s_mb[a];
        if (b < 0) continue;
        const int q0 = OA[a], q1 = OA[a + 1], c0 = OB[b], nc = OB[b + 1] - c0;
        if (nc <= 0) continue;
        if (BOW_BATCH4 && nc <= 16) {
            // Four queries per step, lane 16g + c: query g of the step against candidate c (each
            // of the four 16-lane rows holds the node's candidates and their matched flags).  A
            // query's outcome is fixed by its best and second unmatched candidates and an
            // acceptance marks exactly one candidate, so the step's queries are decided from the
            // step-start state unless an earlier query of the step accepted one of them (the
            // speculation of k_resolve / k_match_init): the step commits its queries before the
            // first such one, at least one per step.
            const int c = lane & 15, g = lane >> 4;
            int myIdx = 0;
            uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
            bool myTaken = true;
            if (c < nc) {
                myIdx = min((unsigned)FB[c0 + c], (unsigned)(nB - 1));
                m0 = DB[2 * (size_t)myIdx];
                m1 = DB[2 * (size_t)myIdx + 1];
                myTaken = s_taken[myIdx] != 0;
            }
            int qIdx = 0, qOk = 0, base = q0 - 64;
            uint4 qd0 = make_uint4(0, 0, 0, 0), qd1 = qd0;
            for (int q = q0; q < q1;) {
                if (q + 4 > base + 64) {  // the next 64 queries, one per lane
                    base = q;
                    qOk = 0;
                    if (q + lane < q1) {
                        qIdx = FA[q + lane];
                        qOk = (unsigned)qIdx < (unsigned)nA && (!UA || UA[qIdx]);  // !pMP || pMP->isBad()
                        const int qi = qOk ? qIdx : 0;
                        qd0 = DA[2 * (size_t)qi];
                        qd1 = DA[2 * (size_t)qi + 1];
                    }
                }
                const int src = q - base + g;  // < 64
                // (every lane takes part in each ds_bpermute: a lane that is inactive for one
                // provides no source data, so none of these sits behind a per-lane condition)
                const int okS = __shfl(qOk, src, 64);
                const bool okG = q + g < q1 && okS != 0;
                uint4 d0, d1;
                d0.x = (uint32_t)__shfl((int)qd0.x, src, 64), d0.y = (uint32_t)__shfl((int)qd0.y, src, 64);
                d0.z = (uint32_t)__shfl((int)qd0.z, src, 64), d0.w = (uint32_t)__shfl((int)qd0.w, src, 64);
                d1.x = (uint32_t)__shfl((int)qd1.x, src, 64), d1.y = (uint32_t)__shfl((int)qd1.y, src, 64);
                d1.z = (uint32_t)__shfl((int)qd1.z, src, 64), d1.w = (uint32_t)__shfl((int)qd1.w, src, 64);
                const uint32_t key = okG && !myTaken ? ((uint32_t)ham(d0, d1, m0, m1) << 16) | (uint32_t)c : NONE;
                const uint32_t b1 = rmin16(key);
                const uint32_t b2 = rmin16(key == b1 ? NONE : key);
                bool accept = false;
                if (b1 != NONE) {
                    const int dist1 = (int)(b1 >> 16);
                    const int dist2 = b2 == NONE ? INT_MAX : (int)(b2 >> 16);
                    const bool thOk = J.kfkf ? dist1 < TH_LOW : dist1 <= TH_LOW;
                    accept = thOk && (float)dist1 < J.nnratio * (float)dist2;
                }
                const int bc = b1 != NONE ? (int)(b1 & 0xFFFFu) : -1, sc = b2 != NONE ? (int)(b2 & 0xFFFFu) : -2;
                const uint64_t accM = __ballot(accept && c == 0);  // bit 16g: query g accepts
                int bcG[4];
#pragma unroll
                for (int h = 0; h < 4; ++h) bcG[h] = __builtin_amdgcn_readlane(bc, 16 * h);
                bool hit = false;
#pragma unroll
                for (int h = 0; h < 3; ++h)
                    hit |= h < g && ((accM >> (16 * h)) & 1ull) && (bcG[h] == bc || bcG[h] == sc);
                const uint64_t stopM = __ballot(hit && c == 0);
                const int nb = min(4, q1 - q);
                const int jstop = stopM ? min((__ffsll((unsigned long long)stopM) - 1) >> 4, nb) : nb;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    if (h >= jstop || !((accM >> (16 * h)) & 1ull)) continue;  // (wave-uniform)
                    if (c == bcG[h]) myTaken = true;
                    if (lane == 0) {
                        const int idx1 = __builtin_amdgcn_readlane(qIdx, q - base + h);
                        const int idx2 = __builtin_amdgcn_readlane(myIdx, bcG[h]);
                        if (J.kfkf)
                            out[idx1] = idx2;
                        else
                            out[idx2] = idx1;
                        ++acc;
                    }
                }
                q += jstop;
            }
            continue;
        }
        const bool small = nc <= 64;
        // <= 64 candidates: one per lane, descriptor held for the whole node
        int myIdx = 0;
        uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
        bool myTaken = true;  // the lane's candidate matched (or unusable): a node's own state, in a register
        if (small && lane < nc) {
            myIdx = min((unsigned)FB[c0 + lane], (unsigned)(nB - 1));  // (clamped: never outside the frame)
            m0 = DB[2 * (size_t)myIdx];
            m1 = DB[2 * (size_t)myIdx + 1];
            myTaken = s_taken[myIdx] != 0;
        }
        // the node's queries 64 at a time: lane j loads query j's index, flag and descriptor (one
        // round trip per 64 queries), each query then takes them by v_readlane
        int qIdx = 0, qOk = 0;
        uint4 qd0 = make_uint4(0, 0, 0, 0), qd1 = qd0;
        for (int q = q0; q < q1; ++q) {
            const int j = (q - q0) & 63;
            if (j == 0) {
                qOk = 0;
                if (q + lane < q1) {
                    qIdx = FA[q + lane];
                    // (an index outside the frame is never produced by transform; skipped)
                    qOk = (unsigned)qIdx < (unsigned)nA && (!UA || UA[qIdx]);  // !pMP || pMP->isBad()
                    const int qi = qOk ? qIdx : 0;
                    qd0 = DA[2 * (size_t)qi];
                    qd1 = DA[2 * (size_t)qi + 1];
                }
            }
            if (!__builtin_amdgcn_readlane(qOk, j)) continue;
            const int idx1 = __builtin_amdgcn_readlane(qIdx, j);
            uint4 d0, d1;
            d0.x = __builtin_amdgcn_readlane(qd0.x, j), d0.y = __builtin_amdgcn_readlane(qd0.y, j);
            d0.z = __builtin_amdgcn_readlane(qd0.z, j), d0.w = __builtin_amdgcn_readlane(qd0.w, j);
            d1.x = __builtin_amdgcn_readlane(qd1.x, j), d1.y = __builtin_amdgcn_readlane(qd1.y, j);
            d1.z = __builtin_amdgcn_readlane(qd1.z, j), d1.w = __builtin_amdgcn_readlane(qd1.w, j);
            uint32_t k1 = NONE, k2 = NONE;  // this lane's two smallest keys
            if (small) {
                if (!myTaken) k1 = ((uint32_t)ham(d0, d1, m0, m1) << 16) | (uint32_t)lane;
            } else {
                for (int j = lane; j < nc; j += 64) {
                    const int idx2 = FB[c0 + j];
                    if ((unsigned)idx2 >= (unsigned)nB || s_taken[idx2]) continue;
                    const uint32_t key =
                        ((uint32_t)ham(d0, d1, DB[2 * (size_t)idx2], DB[2 * (size_t)idx2 + 1]) << 16) | (uint32_t)j;
                    if (key < k1) {
                        k2 = k1;
                        k1 = key;
                    } else if (key < k2) {
                        k2 = key;
                    }
                }
            }
            const uint32_t b1 = wmin(k1);
            if (b1 == NONE) continue;  // bestDist1 stays INT_MAX
            const uint32_t b2 = wmin(k1 == b1 ? k2 : k1);
            const int dist1 = (int)(b1 >> 16);
            const int dist2 = b2 == NONE ? INT_MAX : (int)(b2 >> 16);
            const bool thOk = J.kfkf ? dist1 < TH_LOW : dist1 <= TH_LOW;
            if (!(thOk && (float)dist1 < J.nnratio * (float)dist2)) continue;
            const int jb = (int)(b1 & 0xFFFFu);
            const int idx2 = small ? __builtin_amdgcn_readlane(myIdx, jb) : FB[c0 + jb];
            if (small) {
                if (lane == jb) myTaken = true;  // (a candidate is in exactly one node)
            } else if (lane == 0) {
                s_taken[idx2] = 1;
            }
            if (lane == 0) {
                if (J.kfkf)
                    out[idx1] = idx2;  // vpMatches12[idx1] = vpMapPoints2[bestIdx2]
                else
                    out[idx2] = idx1;  // vpMapPointMatches[bestIdxF] = pMP (the KF feature)
                ++acc;
            }
            // (large nodes) lane 0's LDS write lands before any lane's next read (same wave, in order)
            if (!small) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (lane == 0 && acc) atomicAdd(&s_acc, acc);
    __syncthreads();  // (also orders the output writes before the histogram / removal passes read them)
    if (J.checkOri) {
        // rotHist (ORBmatcher.cc:230-236 / 799-805) from the accepted pairs: an accepted pair is
        // never revisited, so the outputs are exactly the pairs pushed into the histogram (built
        // here in parallel, not by one lane per accept behind two dependent keypoint loads)
        for (int i = tid; i < nOut; i += BOW_T) {
            const int v = out[i];
            if (v >= 0)
                atomicAdd(&s_hist[J.kfkf ? rot_bin(KA[i].angle, KB[v].angle) : rot_bin(KA[v].angle, KB[i].angle)], 1);
        }
        __syncthreads();
        if (tid == 0) {  // ComputeThreeMaxima (ORBmatcher.cc:1748-1789)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO; ++i) {
                const int sz = s_hist[i];
                if (sz > max1) {
                    max3 = max2, max2 = max1, max1 = sz;
                    ind3 = ind2, ind2 = ind1, ind1 = i;
                } else if (sz > max2) {
                    max3 = max2, max2 = sz;
                    ind3 = ind2, ind2 = i;
                } else if (sz > max3) {
                    max3 = sz, ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1, ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
            s_ind[0] = ind1, s_ind[1] = ind2, s_ind[2] = ind3;
        }
        __syncthreads();
        int rem = 0;
        for (int i = tid; i < nOut; i += BOW_T) {
            const int v = out[i];
            if (v < 0) continue;
            const int bin = J.kfkf ? rot_bin(KA[i].angle, KB[v].angle) : rot_bin(KA[v].angle, KB[i].angle);
            if (bin != s_ind[0] && bin != s_ind[1] && bin != s_ind[2]) {
                out[i] = -1;
                ++rem;
            }
        }
        if (rem) atomicAdd(&s_rem, rem);
        __syncthreads();
    }
    if (tid == 0) J.nmatches[p] = s_acc - s_rem;
}

}  // namespace

extern "C" int orb_search_by_bow_batch_device(int kf_kf, const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                              const int32_t* d_counts, int cap, const uint32_t* d_fv_nodes,
                                              const int32_t* d_fv_offsets, const int32_t* d_fv_features,
                                              const int32_t* d_fv_n, int P, const int32_t* d_pair_a,
                                              const int32_t* d_pair_b, const uint8_t* d_usable, float nnratio,
                                              int check_ori, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    if (P < 0 || cap <= 0 || cap > 8192 || (kf_kf != 0 && kf_kf != 1))
        return orb_internal_set_error(ORB_EINVAL, "bad arguments");
    if (P == 0) return ORB_OK;
    if (!d_kps || !d_desc || !d_counts || !d_fv_nodes || !d_fv_offsets || !d_fv_features || !d_fv_n || !d_pair_a ||
        !d_pair_b || !d_match || !d_nmatches)
        return orb_internal_set_error(ORB_EINVAL, "bad arguments");
    if (((uintptr_t)d_desc & 15) != 0) return orb_internal_set_error(ORB_EINVAL, "descriptors must be 16-B aligned");
    BowBatch J{d_kps, d_desc, d_counts, d_fv_nodes, d_fv_offsets, d_fv_features, d_fv_n, d_pair_a, d_pair_b,
               d_usable, d_match, d_nmatches, cap, kf_kf, check_ori ? 1 : 0, nnratio};
    // both frames staged in LDS where they fit (cap <= ~1870 keypoints per frame)
    const size_t ldsStage = bow_stage_bytes(cap);
    static std::once_flag attrOnce;
    std::call_once(attrOnce, [] {
        (void)hipFuncSetAttribute((const void*)k_bow_pairs<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024);
        (void)hipGetLastError();
    });
    if (ldsStage <= 159 * 1024)
        hipLaunchKernelGGL(k_bow_pairs<true>, dim3(P), dim3(BOW_T), ldsStage, (hipStream_t)stream, J);
    else
        hipLaunchKernelGGL(k_bow_pairs<false>, dim3(P), dim3(BOW_T), 5 * (size_t)cap, (hipStream_t)stream, J);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return orb_internal_set_error(ORB_EDEVICE, std::string("k_bow_pairs: ") + hipGetErrorString(e));
    return ORB_OK;
}
