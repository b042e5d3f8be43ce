// orb_oracle_voc.cpp — TEST INFRASTRUCTURE ONLY (CPU parity checker; the product never links it).
//
// Restatement of the DBoW2 vocabulary path ORB-SLAM runs per keyframe / relocalisation frame
// (Frame::ComputeBoW, reference src/Frame.cc:280-287; KeyFrame::ComputeBoW, KeyFrame.cc:56-65):
//   TemplatedVocabulary::loadFromTextFile   Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
//   TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup)       1126-1194
//   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)            1217-1259
//   BowVector::addWeight / addIfNotExist / normalize   Thirdparty/DBoW2/DBoW2/BowVector.cpp:34-84
//   FeatureVector::addFeature                          Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45
//   FORB::distance / fromString                        Thirdparty/DBoW2/DBoW2/FORB.cpp:81-101, 120-135
//   ScoringObject mustNormalize table                  Thirdparty/DBoW2/DBoW2/ScoringObject.h:51-87
// Containers are the reference's own (std::map), so iteration order and summation order are
// the reference's by construction.  DBoW2 is built -O3 -march=native
// (Thirdparty/DBoW2/CMakeLists.txt:5): the L2 accumulation `norm += v*v` (BowVector.cpp:75)
// contracts to fma(v, v, norm) there, written explicitly below; nothing else on the path has
// a contractible shape.
//
// Two reference behaviours are undefined and therefore not restated:
//  * loadFromTextFile's `while(!f.eof()) getline` turns a trailing newline into an extra root
//    child whose descriptor bytes are never written (FORB::fromString parses nothing into a
//    fresh cv::Mat); blank lines are skipped here and in the product.
//  * a leaf reached above level m_L - levelsup leaves the caller's `nid` unwritten
//    (TemplatedVocabulary.h:1251-1252); here and in the product nid = that leaf.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "orb_oracle.h"

namespace {

enum { TF_IDF = 0, TF = 1, IDF = 2, BINARY = 3 };
enum { L1_NORM = 0, L2_NORM = 1, CHI_SQUARE = 2, KL = 3, BHATTACHARYYA = 4, DOT_PRODUCT = 5 };

struct Node {
    uint32_t id = 0;
    double weight = 0;
    std::vector<uint32_t> children;
    uint32_t parent = 0;
    uint32_t word_id = 0;
    uint8_t descriptor[32] = {0};
    bool isLeaf() const { return children.empty(); }
};

int hamming(const uint8_t* a, const uint8_t* b) {  // FORB::distance, FORB.cpp:81-101
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24;
    }
    return dist;
}

}  // namespace

struct oracle_vocabulary {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<Node> nodes;
    std::vector<uint32_t> words;  // word id -> node id

    // TemplatedVocabulary.h:1217-1259
    void transform1(const uint8_t* f, uint32_t& word_id, double& weight, uint32_t* nid, int levelsup) const {
        const int nid_level = L - levelsup;
        if (nid_level <= 0 && nid != nullptr) *nid = 0;
        uint32_t final_id = 0;
        int current_level = 0;
        bool nid_set = nid_level <= 0;
        do {
            ++current_level;
            const std::vector<uint32_t>& ch = nodes[final_id].children;
            final_id = ch[0];
            double best_d = hamming(f, nodes[final_id].descriptor);
            for (size_t j = 1; j < ch.size(); ++j) {
                const double d = hamming(f, nodes[ch[j]].descriptor);
                if (d < best_d) {
                    best_d = d;
                    final_id = ch[j];
                }
            }
            if (nid != nullptr && current_level == nid_level) {
                *nid = final_id;
                nid_set = true;
            }
        } while (!nodes[final_id].isLeaf());
        if (nid != nullptr && !nid_set) *nid = final_id;  // reference: unwritten (see header)
        word_id = nodes[final_id].word_id;
        weight = nodes[final_id].weight;
    }
};

extern "C" {

oracle_vocabulary_t* oracle_vocabulary_load_text(const char* path) {
    // TemplatedVocabulary.h:1338-1424
    std::ifstream f(path);
    if (!f.is_open() || f.eof()) return nullptr;
    auto* v = new oracle_vocabulary();
    std::string s;
    std::getline(f, s);
    std::stringstream ss;
    ss << s;
    int n1 = -1, n2 = -1;
    ss >> v->k >> v->L >> n1 >> n2;
    if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
        delete v;
        return nullptr;
    }
    v->scoring = n1;
    v->weighting = n2;
    v->nodes.resize(1);
    v->nodes[0].id = 0;
    while (std::getline(f, s)) {
        if (s.find_first_not_of(" \t\r") == std::string::npos) continue;  // see header
        std::stringstream ssnode;
        ssnode << s;
        const uint32_t nid = (uint32_t)v->nodes.size();
        v->nodes.resize(v->nodes.size() + 1);
        v->nodes[nid].id = nid;
        int pid = 0;
        ssnode >> pid;
        if (pid < 0 || (uint32_t)pid >= nid) {  // the reference indexes m_nodes[pid] unchecked
            delete v;
            return nullptr;
        }
        v->nodes[nid].parent = (uint32_t)pid;
        v->nodes[pid].children.push_back(nid);
        int nIsLeaf = 0;
        ssnode >> nIsLeaf;
        std::stringstream ssd;
        for (int iD = 0; iD < 32; iD++) {
            std::string e;
            ssnode >> e;
            ssd << e << " ";
        }
        {  // FORB::fromString, FORB.cpp:120-135
            std::stringstream sd(ssd.str());
            for (int i = 0; i < 32; ++i) {
                int n;
                sd >> n;
                if (!sd.fail()) v->nodes[nid].descriptor[i] = (uint8_t)n;
            }
        }
        ssnode >> v->nodes[nid].weight;
        if (nIsLeaf > 0) {
            const uint32_t wid = (uint32_t)v->words.size();
            v->words.push_back(nid);
            v->nodes[nid].word_id = wid;
        }
    }
    return v;
}

oracle_vocabulary_t* oracle_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes,
                                              const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc,
                                              const double* weight) {
    // the tree the text loader builds from the lines (parent, isLeaf, desc, weight), i = 1..n
    auto* v = new oracle_vocabulary();
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->nodes.resize(1);
    for (int i = 0; i < n_nodes; ++i) {
        const uint32_t nid = (uint32_t)v->nodes.size();
        if (parent[i] < 0 || (uint32_t)parent[i] >= nid) {
            delete v;
            return nullptr;
        }
        v->nodes.resize(nid + 1);
        Node& n = v->nodes[nid];
        n.id = nid;
        n.parent = (uint32_t)parent[i];
        std::memcpy(n.descriptor, desc + 32 * (size_t)i, 32);
        n.weight = weight[i];
        if (is_leaf[i]) {
            n.word_id = (uint32_t)v->words.size();
            v->words.push_back(nid);
        }
        v->nodes[parent[i]].children.push_back(nid);
    }
    return v;
}

void oracle_vocabulary_destroy(oracle_vocabulary_t* v) { delete v; }

int oracle_vocabulary_info(const oracle_vocabulary_t* v, int32_t* info) {
    info[0] = v->k;
    info[1] = v->L;
    info[2] = v->scoring;
    info[3] = v->weighting;
    info[4] = (int32_t)v->nodes.size();
    info[5] = (int32_t)v->words.size();
    return 0;
}

int oracle_vocabulary_transform_one(const oracle_vocabulary_t* v, const uint8_t* desc, int levelsup, uint32_t* word,
                                    double* weight, uint32_t* nid) {
    if (v->words.empty()) return -22;
    v->transform1(desc, *word, *weight, nid, levelsup);
    return 0;
}

// TemplatedVocabulary::transform(features, v, fv, levelsup), TemplatedVocabulary.h:1126-1194,
// flattened: BowVector -> (bow_words, bow_values)[*bow_n] in map order; FeatureVector ->
// CSR (fv_nodes[*fv_n], fv_offsets[*fv_n + 1], fv_features).
int oracle_vocabulary_transform(const oracle_vocabulary_t* v, const uint8_t* desc, int n, int levelsup,
                                uint32_t* bow_words, double* bow_values, int* bow_n, uint32_t* fv_nodes,
                                int32_t* fv_offsets, int32_t* fv_features, int* fv_n) {
    std::map<uint32_t, double> bow;                // DBoW2::BowVector
    std::map<uint32_t, std::vector<unsigned>> fv;  // DBoW2::FeatureVector
    *bow_n = 0;
    *fv_n = 0;
    fv_offsets[0] = 0;
    if (v->words.empty()) return 0;
    // mustNormalize (ScoringObject.h:72-87): every scoring but DOT_PRODUCT; L2 only for L2_NORM
    const bool must = v->scoring != DOT_PRODUCT;
    const bool l2 = v->scoring == L2_NORM;
    const bool tf = v->weighting == TF || v->weighting == TF_IDF;
    for (int i = 0; i < n; ++i) {
        uint32_t id, nid = 0;
        double w;
        v->transform1(desc + 32 * (size_t)i, id, w, &nid, levelsup);
        if (w > 0) {
            auto vit = bow.lower_bound(id);
            if (tf) {  // BowVector::addWeight
                if (vit != bow.end() && !(id < vit->first))
                    vit->second += w;
                else
                    bow.insert(vit, std::make_pair(id, w));
            } else {  // BowVector::addIfNotExist
                if (vit == bow.end() || id < vit->first) bow.insert(vit, std::make_pair(id, w));
            }
            fv[nid].push_back((unsigned)i);  // FeatureVector::addFeature
        }
    }
    if (tf && !bow.empty() && !must) {
        const double nd = bow.size();
        for (auto& e : bow) e.second /= nd;
    }
    if (must) {  // BowVector::normalize, BowVector.cpp:62-84
        double norm = 0.0;
        if (!l2) {
            for (auto& e : bow) norm += std::fabs(e.second);
        } else {
            for (auto& e : bow) norm = std::fma(e.second, e.second, norm);
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& e : bow) e.second /= norm;
    }
    int k = 0;
    for (auto& e : bow) {
        bow_words[k] = e.first;
        bow_values[k] = e.second;
        ++k;
    }
    *bow_n = k;
    k = 0;
    int off = 0;
    for (auto& e : fv) {
        fv_nodes[k] = e.first;
        for (unsigned f : e.second) fv_features[off++] = (int32_t)f;
        fv_offsets[++k] = off;
    }
    *fv_n = k;
    return 0;
}

}  // extern "C"
