// orb_voc.hip — the DBoW2 ORB vocabulary on the GPU (part of liborb_hip.so).
//
// Replaces, for the reference's ORBVocabulary (= DBoW2::TemplatedVocabulary<FORB::TDescriptor,
// FORB>, include/ORBVocabulary.h):
//   loadFromTextFile                      Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
//   transform(features, BowVector, FeatureVector, levelsup)                           1126-1194
//   transform(feature, word_id, weight, nid, levelsup)                                1217-1259
// with BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84) and
// FeatureVector::addFeature (FeatureVector.cpp:31-45) — the call Frame::ComputeBoW and
// KeyFrame::ComputeBoW make per frame (src/Frame.cc:280-287, src/KeyFrame.cc:56-65).
//
//   k_voc_descend  16 lanes per descriptor.  At every tree level the lanes score the current
//                  node's children — their descriptors are stored contiguously per parent, so a
//                  level is one coalesced read of k x 32 B — and min-reduce (distance << 16 |
//                  child rank): the reference's strict `d < best_d` keeps the first child of
//                  equal distance.  Out: word id, weight and the node at level L - levelsup.
//   k_voc_bow      one workgroup per frame: BowVector (std::map<WordId, double>) and
//                  FeatureVector (std::map<NodeId, vector<unsigned>>) in map order, from
//                  (key << 32 | feature index) pairs bitonic-sorted in LDS.  Per-word weights are
//                  summed in feature order and the norm accumulated in word order by one lane,
//                  so every double is the reference's, bit for bit.
// Layout in HBM (per vocabulary): child-slot descriptors (32 B per non-root node, grouped by
// parent), child-slot -> node id, node -> {first slot, #children}, node -> word id, weight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orb_abi.h"
#include "orb_device.h"
#include "orb_internal.h"

namespace {

enum { kTF_IDF = 0, kTF = 1, kIDF = 2, kBINARY = 3 };
enum { kL1_NORM = 0, kL2_NORM = 1, kDOT_PRODUCT = 5 };

#define VOC_GROUP 16            // lanes per descriptor in k_voc_descend
#define VOC_MAX_FEATURES 8192   // per-frame capacity of k_voc_bow (keys + values in LDS)

struct VocDev {
    const uint4* slotDesc;     // child slot -> descriptor (2 x uint4)
    const uint4* slotInfo;     // child slot -> {node id, its first child slot, its number of children, 0}
    int2 root;                 // the root's {first child slot, number of children}
    const uint32_t* wordId;    // node -> word id (0 for a non-word, as DBoW2's Node())
    const double* weight;      // node -> weight
    int maxDepth;              // tree height (bounds the descent)
};

// transform(feature, word_id, weight, &nid, levelsup) for descriptors f = 0 .. total-1
// (frame f / cap, row f % cap; rows >= counts[frame] are skipped when counts != NULL).
__global__ void __launch_bounds__(256) k_voc_descend(VocDev V, const uint8_t* __restrict__ desc,
                                                     const int* __restrict__ counts, int cap, long long total,
                                                     int nidLevel, uint32_t* __restrict__ word,
                                                     double* __restrict__ weight, uint32_t* __restrict__ nid) {
    const int sub = threadIdx.x & (VOC_GROUP - 1);
    const long long f = (long long)blockIdx.x * (256 / VOC_GROUP) + (threadIdx.x / VOC_GROUP);
    if (f >= total) return;  // uniform within a 16-lane group
    if (counts) {
        const long long b = f / cap;
        if ((int)(f - b * cap) >= counts[b]) return;
    }
    const uint4* q = (const uint4*)(desc + f * 32);
    const uint4 q0 = q[0], q1 = q[1];
    uint32_t node = 0, nodeAt = 0;  // nid_level <= 0 -> the root (TemplatedVocabulary.h:1227)
    bool set = nidLevel <= 0;
    int2 inf = V.root;
    for (int level = 1;; ++level) {
        uint32_t best = 0xFFFFFFFFu;
        for (int j = sub; j < inf.y; j += VOC_GROUP) {
            const uint4 a = V.slotDesc[2 * (inf.x + j)], c = V.slotDesc[2 * (inf.x + j) + 1];
            const int d = __popc(q0.x ^ a.x) + __popc(q0.y ^ a.y) + __popc(q0.z ^ a.z) + __popc(q0.w ^ a.w) +
                          __popc(q1.x ^ c.x) + __popc(q1.y ^ c.y) + __popc(q1.z ^ c.z) + __popc(q1.w ^ c.w);
            best = min(best, ((uint32_t)d << 16) | (uint32_t)j);
        }
        // min over the 16-lane group (a DPP row): no LDS round trip
        best = orbdev::min8(best);
        best = min(best, (uint32_t)__builtin_amdgcn_update_dpp((int)best, (int)best, 0x140, 0xf, 0xf, false));
        // the chosen child's node and its children in one load (one dependent round trip per level)
        const uint4 si = V.slotInfo[inf.x + (int)(best & 0xFFFFu)];
        node = si.x;
        if (level == nidLevel) {
            nodeAt = node;
            set = true;
        }
        inf = make_int2((int)si.y, (int)si.z);
        if (inf.y == 0 || level >= V.maxDepth) break;  // isLeaf() (TemplatedVocabulary.h:1254)
    }
    if (sub == 0) {
        word[f] = V.wordId[node];
        weight[f] = V.weight[node];
        nid[f] = set ? nodeAt : node;  // a leaf above nid_level: the leaf (reference: unwritten)
    }
}

__device__ void bitonic_sort_u64(uint64_t* s, int P, int tid) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    if ((a > b) == ((i & k) == 0)) {
                        s[i] = b;
                        s[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// Heads of the runs of equal high words among the valid (!= ~0) sorted keys: each thread
// owns a contiguous chunk; s_cnt[t] = heads before chunk t, s_cnt[256] = all heads,
// s_cnt[257] = valid keys (s_cnt[258 ..] is scratch).
__device__ void run_heads(const uint64_t* s_key, int P, int tid, int* s_cnt) {
    const int C = P / 256, i0 = tid * C;
    int heads = 0, valid = 0;
    for (int i = i0; i < i0 + C; ++i) {
        const uint64_t k = s_key[i];
        if (k == ~0ull) continue;
        ++valid;
        if (i == 0 || (s_key[i - 1] >> 32) != (k >> 32)) ++heads;
    }
    s_cnt[tid] = heads;
    s_cnt[258 + tid] = valid;
    __syncthreads();
    if (tid == 0) {
        int s = 0, v = 0;
        for (int t = 0; t < 256; ++t) {
            const int c = s_cnt[t];
            s_cnt[t] = s;
            s += c;
            v += s_cnt[258 + t];
        }
        s_cnt[256] = s;
        s_cnt[257] = v;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_voc_bow(const uint32_t* __restrict__ word, const double* __restrict__ weight,
                                                 const uint32_t* __restrict__ nid, const int* __restrict__ counts,
                                                 int cap, int P, int scoring, int weighting,
                                                 uint32_t* __restrict__ bowW, double* __restrict__ bowV,
                                                 int* __restrict__ bowN, uint32_t* __restrict__ fvNodes,
                                                 int* __restrict__ fvOff, int* __restrict__ fvFeat,
                                                 int* __restrict__ fvN) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint64_t* s_key = (uint64_t*)smem;     // P sort keys
    double* s_val = (double*)(s_key + P);  // per-word values, map order
    __shared__ int s_cnt[258 + 256];
    __shared__ double s_norm;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = min(counts[b], cap);
    const long long base = (long long)b * cap;
    const int C = P / 256, i0 = tid * C;
    const bool tf = weighting == kTF || weighting == kTF_IDF;
    const bool must = scoring != kDOT_PRODUCT;  // mustNormalize, ScoringObject.h:72-87
    // ---- BowVector: features with w > 0 by (word, index) ----
    for (int i = tid; i < P; i += 256)
        s_key[i] = (i < n && weight[base + i] > 0.0) ? (((uint64_t)word[base + i] << 32) | (uint32_t)i) : ~0ull;
    __syncthreads();
    bitonic_sort_u64(s_key, P, tid);
    run_heads(s_key, P, tid, s_cnt);
    {
        int u = s_cnt[tid];
        for (int i = i0; i < i0 + C; ++i) {
            const uint64_t k = s_key[i];
            if (k == ~0ull || (i > 0 && (s_key[i - 1] >> 32) == (k >> 32))) continue;
            double v = weight[base + (uint32_t)k];
            if (tf)  // addWeight: v[id] += w in feature order; IDF/BINARY keep the first (addIfNotExist)
                for (int j = i + 1; j < P && s_key[j] != ~0ull && (s_key[j] >> 32) == (k >> 32); ++j)
                    v += weight[base + (uint32_t)s_key[j]];
            s_val[u] = v;
            bowW[base + u] = (uint32_t)(k >> 32);
            ++u;
        }
    }
    __syncthreads();
    const int m = s_cnt[256];
    if (tid == 0) {  // BowVector::normalize (BowVector.cpp:62-84), in map order
        double norm = 0.0;
        if (must) {
            if (scoring == kL2_NORM) {
                for (int k = 0; k < m; ++k) norm = fma(s_val[k], s_val[k], norm);  // g++ -march=native contraction
                norm = sqrt(norm);
            } else {
                for (int k = 0; k < m; ++k) norm += fabs(s_val[k]);
            }
        }
        s_norm = norm;
    }
    __syncthreads();
    const double norm = s_norm;
    for (int k = tid; k < m; k += 256) {
        double v = s_val[k];
        if (must) {
            if (norm > 0.0) v /= norm;
        } else if (tf) {
            v /= (double)m;  // TemplatedVocabulary.h:1164-1170
        }
        bowV[base + k] = v;
    }
    if (tid == 0) bowN[b] = m;
    __syncthreads();
    // ---- FeatureVector: the same features by (node, index) ----
    for (int i = tid; i < P; i += 256)
        s_key[i] = (i < n && weight[base + i] > 0.0) ? (((uint64_t)nid[base + i] << 32) | (uint32_t)i) : ~0ull;
    __syncthreads();
    bitonic_sort_u64(s_key, P, tid);
    run_heads(s_key, P, tid, s_cnt);
    const long long ob = (long long)b * (cap + 1);
    {
        int u = s_cnt[tid];
        for (int i = i0; i < i0 + C; ++i) {
            const uint64_t k = s_key[i];
            if (k == ~0ull) continue;
            fvFeat[base + i] = (int)(uint32_t)k;  // valid keys are a sorted prefix
            if (i == 0 || (s_key[i - 1] >> 32) != (k >> 32)) {
                fvNodes[base + u] = (uint32_t)(k >> 32);
                fvOff[ob + u] = i;
                ++u;
            }
        }
    }
    if (tid == 0) {
        fvOff[ob + s_cnt[256]] = s_cnt[257];
        fvN[b] = s_cnt[256];
    }
}

int fail(int code, const std::string& msg) { return orb_internal_set_error(code, msg); }

#define VCHK(expr)                                                                                \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(ORB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int pow2_at_least(int n) {
    int p = 256;
    while (p < n) p <<= 1;
    return p;
}

}  // namespace

struct orb_vocabulary {
    int k = 0, L = 0, scoring = 0, weighting = 0, device = 0;
    int nNodes = 0, nWords = 0, maxDepth = 0;
    uint4* d_slotDesc = nullptr;
    uint4* d_slotInfo = nullptr;
    int2 rootInfo{0, 0};
    uint32_t* d_word = nullptr;
    double* d_weight = nullptr;
    // host entry point: own stream + scratch, one caller at a time
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t* d_scratch = nullptr;
    size_t scratchCap = 0;

    VocDev dev() const { return VocDev{d_slotDesc, d_slotInfo, rootInfo, d_word, d_weight, maxDepth}; }

    void release() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        (void)hipFree(d_slotDesc);
        (void)hipFree(d_slotInfo);
        (void)hipFree(d_word);
        (void)hipFree(d_weight);
        (void)hipFree(d_scratch);
        if (stream) (void)hipStreamDestroy(stream);
    }

    // Nodes 1..n in file order: parent[i], is_leaf[i], desc[32 i], weight[i] describe node i + 1
    // (TemplatedVocabulary.h:1378-1420).  Children keep file order; word ids are assigned in
    // file order to the lines with isLeaf > 0.
    int build(int n, const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc, const double* w) {
        const int N = n + 1;
        std::vector<int> cnt(N, 0), first(N + 1, 0), depth(N, 0), fill(N, 0);
        for (int i = 0; i < n; ++i) {
            const int p = parent[i];
            cnt[p]++;
            depth[i + 1] = depth[p] + 1;
        }
        for (int v = 0; v < N; ++v) first[v + 1] = first[v] + cnt[v];
        std::vector<uint4> sdesc((size_t)std::max(n, 1) * 2);
        std::vector<uint32_t> snode(std::max(n, 1)), wid(N, 0u);
        std::vector<int2> info(N);
        std::vector<double> wt(N, 0.0);
        int words = 0, height = 0;
        for (int i = 0; i < n; ++i) {
            const int p = parent[i], s = first[p] + fill[p]++;
            std::memcpy(&sdesc[2 * (size_t)s], desc + 32 * (size_t)i, 32);
            snode[s] = (uint32_t)(i + 1);
            wt[i + 1] = w[i];
            if (is_leaf[i]) wid[i + 1] = (uint32_t)words++;
            height = std::max(height, depth[i + 1]);
        }
        for (int v = 0; v < N; ++v) info[v] = make_int2(first[v], cnt[v]);
        std::vector<uint4> sinfo(std::max(n, 1));
        for (int s2 = 0; s2 < n; ++s2) {
            const uint32_t nd = snode[s2];
            sinfo[s2] = make_uint4(nd, (uint32_t)info[nd].x, (uint32_t)info[nd].y, 0u);
        }
        rootInfo = info[0];
        nNodes = N;
        nWords = words;
        maxDepth = std::max(height, 1);
        VCHK(hipSetDevice(device));
        VCHK(hipMalloc(&d_slotDesc, sdesc.size() * sizeof(uint4)));
        VCHK(hipMalloc(&d_slotInfo, sinfo.size() * sizeof(uint4)));
        VCHK(hipMalloc(&d_word, (size_t)N * 4));
        VCHK(hipMalloc(&d_weight, (size_t)N * 8));
        VCHK(hipMemcpy(d_slotDesc, sdesc.data(), sdesc.size() * sizeof(uint4), hipMemcpyHostToDevice));
        VCHK(hipMemcpy(d_slotInfo, sinfo.data(), sinfo.size() * sizeof(uint4), hipMemcpyHostToDevice));
        VCHK(hipMemcpy(d_word, wid.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        VCHK(hipMemcpy(d_weight, wt.data(), (size_t)N * 8, hipMemcpyHostToDevice));
        VCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        return ORB_OK;
    }
};

namespace {

int check_header(int k, int L, int scoring, int weighting) {
    // the reference's own acceptance test (TemplatedVocabulary.h:1359)
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3)
        return fail(ORB_EINVAL, "vocabulary: not a correct header (k, L, scoring, weighting)");
    return ORB_OK;
}

int check_device(int device) {
    int ndev = 0;
    VCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(ORB_EINVAL, "device ordinal out of range");
    return ORB_OK;
}

int create_from_arrays(int k, int L, int scoring, int weighting, int n, const int32_t* parent, const uint8_t* is_leaf,
                       const uint8_t* desc, const double* weight, int device, orb_vocabulary_t** out) {
    auto* v = new orb_vocabulary();
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->device = device;
    int st = v->build(n, parent, is_leaf, desc, weight);
    if (st) {
        v->release();
        delete v;
        return st;
    }
    *out = v;
    return ORB_OK;
}

// Validation shared by the device entry points (before any device work).
int check_transform_args(const orb_vocabulary_t* v, const void* d_desc) {
    if (!v) return fail(ORB_EINVAL, "NULL vocabulary");
    if (v->nWords == 0) return fail(ORB_EINVAL, "empty vocabulary");
    if (((uintptr_t)d_desc & 15) != 0) return fail(ORB_EINVAL, "descriptors must be 16-byte aligned");
    return ORB_OK;
}

void launch_descend(const orb_vocabulary_t* v, const uint8_t* d_desc, const int32_t* d_counts, int cap,
                    long long total, int levelsup, uint32_t* d_word, double* d_weight, uint32_t* d_node,
                    hipStream_t st) {
    const long long blocks = (total + (256 / VOC_GROUP) - 1) / (256 / VOC_GROUP);
    hipLaunchKernelGGL(k_voc_descend, dim3((unsigned)blocks), dim3(256), 0, st, v->dev(), d_desc, d_counts, cap,
                       total, v->L - levelsup, d_word, d_weight, d_node);
}

int launch_bow(const orb_vocabulary_t* v, int B, const int32_t* d_counts, int cap, const uint32_t* d_word,
               const double* d_weight, const uint32_t* d_node, uint32_t* d_bow_words, double* d_bow_values,
               int32_t* d_bow_n, uint32_t* d_fv_nodes, int32_t* d_fv_offsets, int32_t* d_fv_features,
               int32_t* d_fv_n, hipStream_t st) {
    const int P = pow2_at_least(cap);
    const size_t lds = (size_t)P * 16;
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)k_voc_bow, hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    });
    hipLaunchKernelGGL(k_voc_bow, dim3(B), dim3(256), lds, st, d_word, d_weight, d_node, d_counts, cap, P,
                       v->scoring, v->weighting, d_bow_words, d_bow_values, d_bow_n, d_fv_nodes, d_fv_offsets,
                       d_fv_features, d_fv_n);
    VCHK(hipGetLastError());
    return ORB_OK;
}

}  // namespace

extern "C" {

int orb_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                          const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                          orb_vocabulary_t** out) {
    if (!out) return fail(ORB_EINVAL, "out is NULL");
    *out = nullptr;
    if (n_nodes < 0 || (n_nodes > 0 && (!parent || !is_leaf || !desc || !weight)))
        return fail(ORB_EINVAL, "bad node arrays");
    int st = check_header(k, L, scoring, weighting);
    if (st) return st;
    for (int i = 0; i < n_nodes; ++i)
        if (parent[i] < 0 || parent[i] > i)
            return fail(ORB_EINVAL,
                        "vocabulary: node " + std::to_string(i + 1) + " has a parent that does not precede it");
    st = check_device(device);
    if (st) return st;
    return create_from_arrays(k, L, scoring, weighting, n_nodes, parent, is_leaf, desc, weight, device, out);
}

int orb_vocabulary_load_text(const char* path, int device, orb_vocabulary_t** out) {
    if (!out || !path) return fail(ORB_EINVAL, "bad arguments");
    *out = nullptr;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(ORB_EINVAL, std::string("cannot open vocabulary file ") + path);
    std::string buf;
    {
        std::vector<char> chunk(1 << 16);
        size_t got;
        while ((got = std::fread(chunk.data(), 1, chunk.size(), fp)) > 0) buf.append(chunk.data(), got);
        std::fclose(fp);
    }
    // header: k L scoring weighting (TemplatedVocabulary.h:1349-1363)
    const char* p = buf.c_str();
    const char* end = p + buf.size();
    const char* eol = (const char*)std::memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    int hdr[4];
    {
        const char* q = p;
        for (int t = 0; t < 4; ++t) {
            char* e = nullptr;
            const long x = std::strtol(q, &e, 10);
            if (e == q || e > eol) return fail(ORB_EINVAL, "vocabulary: not a correct header");
            hdr[t] = (int)x;
            q = e;
        }
    }
    int st = check_header(hdr[0], hdr[1], hdr[2], hdr[3]);
    if (st) return st;
    st = check_device(device);
    if (st) return st;
    // node lines: parent isLeaf d0 .. d31 weight (TemplatedVocabulary.h:1378-1420)
    std::vector<int32_t> parent;
    std::vector<uint8_t> leaf, desc;
    std::vector<double> weight;
    p = eol < end ? eol + 1 : end;
    while (p < end) {
        eol = (const char*)std::memchr(p, '\n', (size_t)(end - p));
        if (!eol) eol = end;
        const char* q = p;
        while (q < eol && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
        if (q == eol) {  // blank line (the reference's trailing-newline node)
            p = eol + 1;
            continue;
        }
        const std::string line = std::to_string(parent.size() + 2);
        char* e = nullptr;
        const long pid = std::strtol(q, &e, 10);
        if (e == q || e > eol) return fail(ORB_EINVAL, "vocabulary: malformed node line " + line);
        q = e;
        const long isLeaf = std::strtol(q, &e, 10);
        if (e == q || e > eol) return fail(ORB_EINVAL, "vocabulary: malformed node line " + line);
        q = e;
        uint8_t d[32];
        for (int i = 0; i < 32; ++i) {
            const long x = std::strtol(q, &e, 10);
            if (e == q || e > eol) return fail(ORB_EINVAL, "vocabulary: malformed node line " + line);
            d[i] = (uint8_t)x;  // FORB::fromString: (unsigned char)n
            q = e;
        }
        const double w = std::strtod(q, &e);  // istream >> double: correctly rounded, as strtod
        if (e == q || e > eol) return fail(ORB_EINVAL, "vocabulary: malformed node line " + line);
        if (pid < 0 || pid > (long)parent.size())
            return fail(ORB_EINVAL, "vocabulary: node line " + line + " names a later parent");
        parent.push_back((int32_t)pid);
        leaf.push_back(isLeaf > 0 ? 1 : 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
        p = eol + 1;
    }
    return create_from_arrays(hdr[0], hdr[1], hdr[2], hdr[3], (int)parent.size(), parent.data(), leaf.data(),
                              desc.data(), weight.data(), device, out);
}

int orb_vocabulary_destroy(orb_vocabulary_t* v) {
    if (!v) return ORB_OK;
    v->release();
    delete v;
    return ORB_OK;
}

int orb_vocabulary_info(const orb_vocabulary_t* v, int32_t* info) {
    if (!v || !info) return fail(ORB_EINVAL, "bad arguments");
    info[0] = v->k;
    info[1] = v->L;
    info[2] = v->scoring;
    info[3] = v->weighting;
    info[4] = v->nNodes;
    info[5] = v->nWords;
    info[6] = v->maxDepth;
    return ORB_OK;
}

int orb_vocabulary_transform_features_device(const orb_vocabulary_t* v, int n, const uint8_t* d_desc, int levelsup,
                                             uint32_t* d_word, double* d_weight, uint32_t* d_node, void* stream) {
    if (n < 0 || (n > 0 && (!d_desc || !d_word || !d_weight || !d_node))) return fail(ORB_EINVAL, "bad arguments");
    int st = check_transform_args(v, d_desc);
    if (st) return st;
    if (n == 0) return ORB_OK;
    VCHK(hipSetDevice(v->device));
    launch_descend(v, d_desc, nullptr, n, n, levelsup, d_word, d_weight, d_node, (hipStream_t)stream);
    VCHK(hipGetLastError());
    return ORB_OK;
}

int orb_vocabulary_transform_batch_device(const orb_vocabulary_t* v, int B, const uint8_t* d_desc,
                                          const int32_t* d_counts, int cap, int levelsup, uint32_t* d_feat_word,
                                          double* d_feat_weight, uint32_t* d_feat_node, uint32_t* d_bow_words,
                                          double* d_bow_values, int32_t* d_bow_n, uint32_t* d_fv_nodes,
                                          int32_t* d_fv_offsets, int32_t* d_fv_features, int32_t* d_fv_n,
                                          void* stream) {
    if (B <= 0 || cap <= 0 || !d_desc || !d_counts || !d_feat_word || !d_feat_weight || !d_feat_node ||
        !d_bow_words || !d_bow_values || !d_bow_n || !d_fv_nodes || !d_fv_offsets || !d_fv_features || !d_fv_n)
        return fail(ORB_EINVAL, "bad arguments");
    if (cap > VOC_MAX_FEATURES) return fail(ORB_ENOTSUP, "more than 8192 features per frame");
    int st = check_transform_args(v, d_desc);
    if (st) return st;
    VCHK(hipSetDevice(v->device));
    const hipStream_t s = (hipStream_t)stream;
    launch_descend(v, d_desc, d_counts, cap, (long long)B * cap, levelsup, d_feat_word, d_feat_weight, d_feat_node,
                   s);
    return launch_bow(v, B, d_counts, cap, d_feat_word, d_feat_weight, d_feat_node, d_bow_words, d_bow_values,
                      d_bow_n, d_fv_nodes, d_fv_offsets, d_fv_features, d_fv_n, s);
}

int orb_vocabulary_transform(orb_vocabulary_t* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                             double* bow_values, int* bow_n, uint32_t* fv_nodes, int32_t* fv_offsets,
                             int32_t* fv_features, int* fv_n) {
    if (!v || n < 0 || !bow_n || !fv_n || !fv_offsets ||
        (n > 0 && (!desc || !bow_words || !bow_values || !fv_nodes || !fv_features)))
        return fail(ORB_EINVAL, "bad arguments");
    if (n > VOC_MAX_FEATURES) return fail(ORB_ENOTSUP, "more than 8192 features");
    *bow_n = 0;
    *fv_n = 0;
    fv_offsets[0] = 0;
    if (v->nWords == 0 || n == 0) return ORB_OK;  // empty(): v.clear(), fv.clear(), return
    std::lock_guard<std::mutex> lock(v->mu);
    VCHK(hipSetDevice(v->device));
    // scratch: desc | word | weight | node | bow words | values | fv nodes | offsets | features | counts | n
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t oDesc = 0, oWord = al(oDesc + (size_t)n * 32), oWt = al(oWord + (size_t)n * 4),
                 oNode = al(oWt + (size_t)n * 8), oBw = al(oNode + (size_t)n * 4), oBv = al(oBw + (size_t)n * 4),
                 oFn = al(oBv + (size_t)n * 8), oFo = al(oFn + (size_t)n * 4), oFf = al(oFo + (size_t)(n + 1) * 4),
                 oCnt = al(oFf + (size_t)n * 4), oN = al(oCnt + 4), total = al(oN + 8);
    if (total > v->scratchCap) {
        (void)hipFree(v->d_scratch);
        v->d_scratch = nullptr;
        v->scratchCap = 0;
        VCHK(hipMalloc(&v->d_scratch, total));
        v->scratchCap = total;
    }
    uint8_t* S = v->d_scratch;
    const hipStream_t st = v->stream;
    const int32_t cnt = n;
    VCHK(hipMemcpyAsync(S + oDesc, desc, (size_t)n * 32, hipMemcpyHostToDevice, st));
    VCHK(hipMemcpyAsync(S + oCnt, &cnt, 4, hipMemcpyHostToDevice, st));
    int r = orb_vocabulary_transform_batch_device(
        v, 1, S + oDesc, (const int32_t*)(S + oCnt), n, levelsup, (uint32_t*)(S + oWord), (double*)(S + oWt),
        (uint32_t*)(S + oNode), (uint32_t*)(S + oBw), (double*)(S + oBv), (int32_t*)(S + oN), (uint32_t*)(S + oFn),
        (int32_t*)(S + oFo), (int32_t*)(S + oFf), (int32_t*)(S + oN + 4), st);
    if (r) return r;
    int32_t nn[2] = {0, 0};
    VCHK(hipMemcpyAsync(nn, S + oN, 8, hipMemcpyDeviceToHost, st));
    VCHK(hipStreamSynchronize(st));
    const int bn = nn[0], fn = nn[1];
    VCHK(hipMemcpyAsync(bow_words, S + oBw, (size_t)bn * 4, hipMemcpyDeviceToHost, st));
    VCHK(hipMemcpyAsync(bow_values, S + oBv, (size_t)bn * 8, hipMemcpyDeviceToHost, st));
    VCHK(hipMemcpyAsync(fv_nodes, S + oFn, (size_t)fn * 4, hipMemcpyDeviceToHost, st));
    VCHK(hipMemcpyAsync(fv_offsets, S + oFo, (size_t)(fn + 1) * 4, hipMemcpyDeviceToHost, st));
    VCHK(hipStreamSynchronize(st));
    const int nfeat = fv_offsets[fn];
    VCHK(hipMemcpyAsync(fv_features, S + oFf, (size_t)nfeat * 4, hipMemcpyDeviceToHost, st));
    VCHK(hipStreamSynchronize(st));
    *bow_n = bn;
    *fv_n = fn;
    return ORB_OK;
}

}  // extern "C"
