/*
 * orb_oracle_match.cpp — TEST INFRASTRUCTURE ONLY (parity checker; never shipped, never
 * called by the product path).  Only tests/ may load it (through liborb_oracle.so).
 *
 * CPU restatement of the rest of the reference's ORBmatcher family and the geometry it
 * calls, written as a reading of (caomw/ORBSLAM_jpMiniPC @ /root/reference):
 *   src/ORBmatcher.cc:49-133    SearchByProjection(Frame&, vector<MapPoint*>, th), RadiusByViewingCos
 *   src/ORBmatcher.cc:136-153   CheckDistEpipolarLine
 *   src/ORBmatcher.cc:286-407   SearchByProjection(KeyFrame*, Scw, ...)
 *   src/ORBmatcher.cc:409-516   WindowSearch
 *   src/ORBmatcher.cc:519-594   SearchByProjection(Frame&, Frame&, windowSize, ...)
 *   src/ORBmatcher.cc:852-1014  SearchForTriangulation
 *   src/ORBmatcher.cc:1016-1265 Fuse (both overloads)
 *   src/ORBmatcher.cc:1267-1505 SearchBySim3
 *   src/ORBmatcher.cc:1507-1746 SearchByProjection(Frame&, const Frame&, th) and (Frame&, KeyFrame*, ...)
 *   src/Frame.cc:137-198        Frame::isInFrustum
 *   src/Frame.cc:200-277        Frame::GetFeaturesInArea, PosInGrid
 *   src/KeyFrame.cc:612-657     KeyFrame::GetFeaturesInArea, IsInImage
 *
 * FP policy.  The reference is built with g++ -O3 -march=native (CMakeLists.txt:13), so GCC
 * contracts some a*b+c in these files into FMAs.  Which product it fuses depends on the
 * compiler, so the contraction is pinned the way orb_oracle.cpp pins rBRIEF's: the
 * reference's expression shapes compiled by g++ 11 -O3 -mavx2 -mfma
 * (scripts/contraction_check.sh prints the asm) and written here as explicit std::fma; this
 * TU is compiled -ffp-contract=off and the HIP kernels use the same explicit fmaf.  cv::Mat arithmetic lives in OpenCV
 * (no FMA in a baseline-x86-64 build) and is restated in ocv_ops.cpp, compiled without
 * contraction.  OpenCV itself is absent here: those semantics are parity-unpinned against a
 * real OpenCV build (DESIGN.md §FP policy).
 */
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orb_oracle.h"
#include "ocv_ops.h"

using namespace std;  // the reference's abs / floor / ceil / round resolve through it

namespace {
const int FRAME_GRID_ROWS = 48, FRAME_GRID_COLS = 64;  // Frame.h:35-36
const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;

inline int dist256(const uint8_t* a8, const uint8_t* b8) {  // ORBmatcher.cc:1794-1810
    const uint32_t* pa = (const uint32_t*)a8;
    const uint32_t* pb = (const uint32_t*)b8;
    int dist = 0;
    for (int i = 0; i < 8; i++, pa++, pb++) {
        unsigned int v = *pa ^ *pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// Frame / KeyFrame feature grid (Frame.cc:73-86, 109-123, 267-277; KeyFrame.cc:43-51 copies it)
struct View {
    const orb_frame_view_t& v;
    float invW, invH;
    std::vector<std::vector<size_t>> grid;
    explicit View(const orb_frame_view_t& fv) : v(fv) {
        invW = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(v.bounds.max_x - v.bounds.min_x);
        invH = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(v.bounds.max_y - v.bounds.min_y);
        grid.assign(FRAME_GRID_COLS * FRAME_GRID_ROWS, {});
        for (int i = 0; i < v.n; ++i) {
            const int posX = round((v.kps[i].x - v.bounds.min_x) * invW);
            const int posY = round((v.kps[i].y - v.bounds.min_y) * invH);
            if (posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS) continue;
            grid[posX * FRAME_GRID_ROWS + posY].push_back(i);
        }
    }
    const uint8_t* desc(size_t i) const { return v.desc + i * 32; }
    // Frame::GetFeaturesInArea (Frame.cc:200-265)
    std::vector<size_t> area(const float& x, const float& y, const float& r, int minLevel, int maxLevel) const {
        std::vector<size_t> vIndices;
        const int mnMinX = v.bounds.min_x, mnMinY = v.bounds.min_y;
        int nMinCellX = floor((x - mnMinX - r) * invW);
        nMinCellX = max(0, nMinCellX);
        if (nMinCellX >= FRAME_GRID_COLS) return vIndices;
        int nMaxCellX = ceil((x - mnMinX + r) * invW);
        nMaxCellX = min(FRAME_GRID_COLS - 1, nMaxCellX);
        if (nMaxCellX < 0) return vIndices;
        int nMinCellY = floor((y - mnMinY - r) * invH);
        nMinCellY = max(0, nMinCellY);
        if (nMinCellY >= FRAME_GRID_ROWS) return vIndices;
        int nMaxCellY = ceil((y - mnMinY + r) * invH);
        nMaxCellY = min(FRAME_GRID_ROWS - 1, nMaxCellY);
        if (nMaxCellY < 0) return vIndices;
        bool bCheckLevels = true, bSameLevel = false;
        if (minLevel == -1 && maxLevel == -1)
            bCheckLevels = false;
        else if (minLevel == maxLevel)
            bSameLevel = true;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const std::vector<size_t>& vCell = grid[ix * FRAME_GRID_ROWS + iy];
                for (size_t j = 0; j < vCell.size(); j++) {
                    const orb_keypoint_t& kpUn = v.kps[vCell[j]];
                    if (bCheckLevels && !bSameLevel) {
                        if (kpUn.octave < minLevel || kpUn.octave > maxLevel) continue;
                    } else if (bSameLevel) {
                        if (kpUn.octave != minLevel) continue;
                    }
                    if (abs(kpUn.x - x) > r || abs(kpUn.y - y) > r) continue;
                    vIndices.push_back(vCell[j]);
                }
            }
        return vIndices;
    }
    // KeyFrame::GetFeaturesInArea (KeyFrame.cc:612-652)
    std::vector<size_t> kf_area(const float& x, const float& y, const float& r) const {
        std::vector<size_t> vIndices;
        const int mnMinX = v.bounds.min_x, mnMinY = v.bounds.min_y;
        int nMinCellX = floor((x - mnMinX - r) * invW);
        nMinCellX = max(0, nMinCellX);
        if (nMinCellX >= FRAME_GRID_COLS) return vIndices;
        int nMaxCellX = ceil((x - mnMinX + r) * invW);
        nMaxCellX = min(FRAME_GRID_COLS - 1, nMaxCellX);
        if (nMaxCellX < 0) return vIndices;
        int nMinCellY = floor((y - mnMinY - r) * invH);
        nMinCellY = max(0, nMinCellY);
        if (nMinCellY >= FRAME_GRID_ROWS) return vIndices;
        int nMaxCellY = ceil((y - mnMinY + r) * invH);
        nMaxCellY = min(FRAME_GRID_ROWS - 1, nMaxCellY);
        if (nMaxCellY < 0) return vIndices;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const std::vector<size_t>& vCell = grid[ix * FRAME_GRID_ROWS + iy];
                for (size_t j = 0; j < vCell.size(); j++) {
                    const orb_keypoint_t& kpUn = v.kps[vCell[j]];
                    if (abs(kpUn.x - x) <= r && abs(kpUn.y - y) <= r) vIndices.push_back(vCell[j]);
                }
            }
        return vIndices;
    }
    // KeyFrame::IsInImage (KeyFrame.cc:654-657)
    bool in_image(const float& x, const float& y) const {
        return (x >= v.bounds.min_x && x < v.bounds.max_x && y >= v.bounds.min_y && y < v.bounds.max_y);
    }
    // lower_bound over mvScaleFactors, clamped to the last level
    int predict_level(float ratio) const {
        const float* sf = v.scale_factors;
        const int n = (int)(std::lower_bound(sf, sf + v.nlevels, ratio) - sf);
        return min(n, v.nlevels - 1);
    }
};

void three_maxima(const std::vector<int>* histo, int& ind1, int& ind2, int& ind3) {  // 1748-1789
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = histo[i].size();
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

// Drop the histogram bins outside the three maxima: out[entry] = -1, nmatches-- per entry.
void rot_filter(std::vector<int>* rotHist, int32_t* out, int& nmatches) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (size_t j = 0; j < rotHist[i].size(); j++) {
            out[rotHist[i][j]] = -1;
            nmatches--;
        }
    }
}

const float* row3(const float* p, int i) { return p + 3 * (size_t)i; }

template <class F>
void fv_walk(const orb_feature_vector_t& f1, const orb_feature_vector_t& f2, F&& body) {
    int a = 0, b = 0;
    while (a < f1.n_nodes && b < f2.n_nodes) {
        if (f1.nodes[a] == f2.nodes[b]) {
            body(a, b);
            ++a;
            ++b;
        } else if (f1.nodes[a] < f2.nodes[b]) {
            a = (int)(std::lower_bound(f1.nodes, f1.nodes + f1.n_nodes, f2.nodes[b]) - f1.nodes);
        } else {
            b = (int)(std::lower_bound(f2.nodes, f2.nodes + f2.n_nodes, f1.nodes[a]) - f2.nodes);
        }
    }
}
}  // namespace

extern "C" {

int oracle_features_in_area_view(const orb_frame_view_t* view, int keyframe, float x, float y, float r, int min_level,
                                 int max_level, int32_t* out, int cap) {
    View V(*view);
    std::vector<size_t> v = keyframe ? V.kf_area(x, y, r) : V.area(x, y, r, min_level, max_level);
    if ((int)v.size() > cap) return ORB_ERANGE;
    for (size_t i = 0; i < v.size(); ++i) out[i] = (int32_t)v[i];
    return (int)v.size();
}

// Frame::isInFrustum (Frame.cc:137-198)
int oracle_frame_is_in_frustum(const orb_frame_view_t* F, orb_map_points_t mps, float viewingCosLimit,
                               uint8_t* in_view, float* proj_x, float* proj_y, int32_t* level, float* view_cos) {
    View V(*F);
    const float fx = F->fx, fy = F->fy, cx = F->cx, cy = F->cy;
    for (int i = 0; i < mps.n; ++i) {
        in_view[i] = 0;
        proj_x[i] = proj_y[i] = 0.f;
        level[i] = -1;
        view_cos[i] = 0.f;
        const float* P = row3(mps.pos, i);
        float Pc[3];
        ocv::gemm3_add(F->Rcw, P, F->tcw, Pc);
        const float PcX = Pc[0];
        const float PcY = Pc[1];
        const float PcZ = Pc[2];
        if (PcZ < 0.0) continue;
        const float invz = 1.0 / PcZ;
        const float u = std::fma(fx * PcX, invz, cx);  // fx*PcX*invz+cx, contracted
        const float v = std::fma(fy * PcY, invz, cy);
        if (u < F->bounds.min_x || u > F->bounds.max_x) continue;
        if (v < F->bounds.min_y || v > F->bounds.max_y) continue;
        const float maxDistance = mps.dmax[i];
        const float minDistance = mps.dmin[i];
        float PO[3];
        ocv::sub3(P, F->Ow, PO);
        const float dist = ocv::norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        float viewCos = ocv::dot3(PO, row3(mps.normal, i)) / dist;
        if (viewCos < viewingCosLimit) continue;
        float ratio = dist / minDistance;
        const float* sf = F->scale_factors;
        int nPredictedLevel = (int)(std::lower_bound(sf, sf + F->nlevels, ratio) - sf);
        if (nPredictedLevel >= F->nlevels) nPredictedLevel = F->nlevels - 1;
        in_view[i] = 1;
        proj_x[i] = u;
        proj_y[i] = v;
        level[i] = nPredictedLevel;
        view_cos[i] = viewCos;
    }
    return ORB_OK;
}

// SearchByProjection(Frame& F, const vector<MapPoint*>&, th) (ORBmatcher.cc:49-125)
int oracle_search_by_projection_local(const orb_frame_view_t* Fv, const uint8_t* f_taken, int n_mp,
                                      const uint8_t* usable, const float* proj_x, const float* proj_y,
                                      const int32_t* level, const float* view_cos, const uint8_t* mp_desc, float th,
                                      float nnratio, int32_t* f_match, int* n_matches) {
    View F(*Fv);
    std::vector<char> taken(f_taken, f_taken + Fv->n);
    for (int j = 0; j < Fv->n; ++j) f_match[j] = -1;
    int nmatches = 0;
    const bool bFactor = th != 1.0;
    for (int iMP = 0; iMP < n_mp; iMP++) {
        if (!usable[iMP]) continue;
        const int& nPredictedLevel = level[iMP];
        float r = view_cos[iMP] > 0.998 ? 2.5 : 4.0;  // RadiusByViewingCos (127-133)
        if (bFactor) r *= th;
        std::vector<size_t> vNearIndices =
            F.area(proj_x[iMP], proj_y[iMP], r * Fv->scale_factors[nPredictedLevel], nPredictedLevel - 1, nPredictedLevel);
        if (vNearIndices.empty()) continue;
        const uint8_t* MPdescriptor = mp_desc + (size_t)iMP * 32;
        int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
        for (size_t idx : vNearIndices) {
            if (taken[idx]) continue;
            const int dist = dist256(MPdescriptor, F.desc(idx));
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = Fv->kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = Fv->kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            taken[bestIdx] = 1;
            f_match[bestIdx] = iMP;
            nmatches++;
        }
    }
    *n_matches = nmatches;
    return ORB_OK;
}

// WindowSearch (ORBmatcher.cc:409-516)
int oracle_window_search(const orb_frame_view_t* F1v, const uint8_t* usable1, const orb_frame_view_t* F2v,
                         int windowSize, int minScaleLevel, int maxScaleLevel, float nnratio, int check_ori,
                         int32_t* match21, int* n_matches) {
    View F2(*F2v);
    int nmatches = 0;
    for (int j = 0; j < F2v->n; ++j) match21[j] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    const bool bMinLevel = minScaleLevel > 0;
    const bool bMaxLevel = maxScaleLevel < INT_MAX;
    for (int i1 = 0; i1 < F1v->n; i1++) {
        if (!usable1[i1]) continue;
        const orb_keypoint_t& kp1 = F1v->kps[i1];
        int level1 = kp1.octave;
        if (bMinLevel)
            if (level1 < minScaleLevel) continue;
        if (bMaxLevel)
            if (level1 > maxScaleLevel) continue;
        std::vector<size_t> vIndices2 = F2.area(kp1.x, kp1.y, windowSize, level1, level1);
        if (vIndices2.empty()) continue;
        const uint8_t* d1 = F1v->desc + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (match21[i2] >= 0) continue;
            int dist = dist256(d1, F2.desc(i2));
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= bestDist2 * nnratio && bestDist <= TH_HIGH) {
            match21[bestIdx2] = i1;
            nmatches++;
            float rot = F1v->kps[i1].angle - F2v->kps[bestIdx2].angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = round(rot * (1.0f / HISTO_LENGTH));
            if (bin == HISTO_LENGTH) bin = 0;
            rotHist[bin].push_back(bestIdx2);
        }
    }
    if (check_ori) rot_filter(rotHist, match21, nmatches);
    *n_matches = nmatches;
    return ORB_OK;
}

// SearchByProjection(Frame& F1, Frame& F2, windowSize, vpMapPointMatches2) (ORBmatcher.cc:519-594)
int oracle_search_by_projection_f2f(const orb_frame_view_t* F1v, orb_map_points_t mp1, const uint8_t* usable1,
                                    const orb_frame_view_t* F2v, const uint8_t* f2_taken, int windowSize,
                                    float nnratio, int32_t* match2, int* n_matches) {
    View F2(*F2v);
    std::vector<char> taken(f2_taken, f2_taken + F2v->n);
    for (int j = 0; j < F2v->n; ++j) match2[j] = -1;
    int nmatches = 0;
    for (int i1 = 0; i1 < F1v->n; i1++) {
        if (!usable1[i1]) continue;
        orb_keypoint_t kp1 = F1v->kps[i1];
        int level1 = kp1.octave;
        float x3Dc2[3];
        ocv::gemm3_add(F2v->Rcw, row3(mp1.pos, i1), F2v->tcw, x3Dc2);
        const float xc2 = x3Dc2[0];
        const float yc2 = x3Dc2[1];
        const float invzc2 = 1.0 / x3Dc2[2];
        float u2 = std::fma(F2v->fx * xc2, invzc2, F2v->cx);
        float v2 = std::fma(F2v->fy * yc2, invzc2, F2v->cy);
        std::vector<size_t> vIndices2 = F2.area(u2, v2, windowSize, level1, level1);
        if (vIndices2.empty()) continue;
        const uint8_t* d1 = F1v->desc + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (taken[i2]) continue;
            int dist = dist256(d1, F2.desc(i2));
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (static_cast<float>(bestDist) <= static_cast<float>(bestDist2) * nnratio && bestDist <= TH_HIGH) {
            taken[bestIdx2] = 1;
            match2[bestIdx2] = i1;
            nmatches++;
        }
    }
    *n_matches = nmatches;
    return ORB_OK;
}

// SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th) (ORBmatcher.cc:1507-1620)
int oracle_search_by_projection_motion(const orb_frame_view_t* Cv, const uint8_t* cur_taken,
                                       const orb_frame_view_t* Lv, orb_map_points_t mp, const uint8_t* usable,
                                       float th, int check_ori, int32_t* cur_match, int* n_matches) {
    View C(*Cv);
    std::vector<char> taken(cur_taken, cur_taken + Cv->n);
    for (int j = 0; j < Cv->n; ++j) cur_match[j] = -1;
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    for (int i = 0; i < Lv->n; i++) {
        if (!usable[i]) continue;
        float x3Dc[3];
        ocv::gemm3_add(Cv->Rcw, row3(mp.pos, i), Cv->tcw, x3Dc);
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        float u = std::fma(Cv->fx * xc, invzc, Cv->cx);
        float v = std::fma(Cv->fy * yc, invzc, Cv->cy);
        if (u < Cv->bounds.min_x || u > Cv->bounds.max_x) continue;
        if (v < Cv->bounds.min_y || v > Cv->bounds.max_y) continue;
        int nPredictedOctave = Lv->kps[i].octave;
        float radius = th * Cv->scale_factors[nPredictedOctave];
        std::vector<size_t> vIndices2 = C.area(u, v, radius, nPredictedOctave - 1, nPredictedOctave + 1);
        if (vIndices2.empty()) continue;
        const uint8_t* dMP = Lv->desc + (size_t)i * 32;
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (taken[i2]) continue;
            int dist = dist256(dMP, C.desc(i2));
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            taken[bestIdx2] = 1;
            cur_match[bestIdx2] = i;
            nmatches++;
            if (check_ori) {
                float rot = Lv->kps[i].angle - Cv->kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = round(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) rot_filter(rotHist, cur_match, nmatches);
    *n_matches = nmatches;
    return ORB_OK;
}

// SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th, ORBdist) (1622-1746)
int oracle_search_by_projection_reloc(const orb_frame_view_t* Cv, const uint8_t* cur_taken,
                                      const orb_frame_view_t* KFv, orb_map_points_t mp, const uint8_t* usable,
                                      float th, int ORBdist, int check_ori, int32_t* cur_match, int* n_matches) {
    View C(*Cv);
    std::vector<char> taken(cur_taken, cur_taken + Cv->n);
    for (int j = 0; j < Cv->n; ++j) cur_match[j] = -1;
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    for (int i = 0; i < KFv->n; i++) {
        if (!usable[i]) continue;
        const float* x3Dw = row3(mp.pos, i);
        float x3Dc[3];
        ocv::gemm3_add(Cv->Rcw, x3Dw, Cv->tcw, x3Dc);
        const float xc = x3Dc[0];
        const float yc = x3Dc[1];
        const float invzc = 1.0 / x3Dc[2];
        float u = std::fma(Cv->fx * xc, invzc, Cv->cx);
        float v = std::fma(Cv->fy * yc, invzc, Cv->cy);
        if (u < Cv->bounds.min_x || u > Cv->bounds.max_x) continue;
        if (v < Cv->bounds.min_y || v > Cv->bounds.max_y) continue;
        float minDistance = mp.dmin[i];
        float PO[3];
        ocv::sub3(x3Dw, Cv->Ow, PO);
        float dist3D = ocv::norm3(PO);
        float ratio = dist3D / minDistance;
        const int nPredictedLevel = C.predict_level(ratio);
        float radius = th * Cv->scale_factors[nPredictedLevel];
        std::vector<size_t> vIndices2 = C.area(u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1);
        if (vIndices2.empty()) continue;
        const uint8_t* dMP = mp.desc + (size_t)i * 32;
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (taken[i2]) continue;
            int dist = dist256(dMP, C.desc(i2));
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= ORBdist) {
            taken[bestIdx2] = 1;
            cur_match[bestIdx2] = i;
            nmatches++;
            if (check_ori) {
                float rot = KFv->kps[i].angle - Cv->kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = round(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) rot_filter(rotHist, cur_match, nmatches);
    *n_matches = nmatches;
    return ORB_OK;
}

// The shared body of SearchByProjection(KF, Scw) (286-407), Fuse(KF, vector) (1016-1134) and
// Fuse(KF, Scw) (1136-1265): project, IsInImage, distance band, viewing angle, predicted
// level, KeyFrame area search, level window [pred-1, pred], best distance.
// `invz_double`: 1.0/z (Fuse(Scw)) vs 1/z (the other two).  Returns bestIdx or -1 (and dist).
static int kf_project_best(const View& K, const float* p3Dw, const float* Pn, float minDistance, float maxDistance,
                           const uint8_t* dMP, float th, bool invz_double, const std::vector<char>* taken,
                           int* bestDistOut) {
    const orb_frame_view_t& kf = K.v;
    const float fx = kf.fx, fy = kf.fy, cx = kf.cx, cy = kf.cy;
    float p3Dc[3];
    ocv::gemm3_add(kf.Rcw, p3Dw, kf.tcw, p3Dc);
    if (p3Dc[2] < 0.0f) return -1;
    float invz;
    if (invz_double)
        invz = 1.0 / p3Dc[2];
    else
        invz = 1 / p3Dc[2];
    const float x = p3Dc[0] * invz;
    const float y = p3Dc[1] * invz;
    const float u = std::fma(fx, x, cx);  // fx*x+cx, contracted
    const float v = std::fma(fy, y, cy);
    if (!K.in_image(u, v)) return -1;
    float PO[3];
    ocv::sub3(p3Dw, kf.Ow, PO);
    const float dist3D = ocv::norm3(PO);
    if (dist3D < minDistance || dist3D > maxDistance) return -1;
    if (ocv::dot3(PO, Pn) < 0.5 * dist3D) return -1;
    const float ratio = dist3D / minDistance;
    const int nPredictedLevel = K.predict_level(ratio);
    const float radius = th * kf.scale_factors[nPredictedLevel];
    std::vector<size_t> vIndices = K.kf_area(u, v, radius);
    if (vIndices.empty()) return -1;
    int bestDist = INT_MAX, bestIdx = -1;
    for (size_t idx : vIndices) {
        if (taken && (*taken)[idx]) continue;
        const int kpLevel = kf.kps[idx].octave;
        if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
        const int dist = dist256(dMP, K.desc(idx));
        if (dist < bestDist) {
            bestDist = dist;
            bestIdx = idx;
        }
    }
    *bestDistOut = bestDist;
    return bestIdx;
}

int oracle_search_by_projection_sim3(const orb_frame_view_t* KFv, const uint8_t* kf_taken, orb_map_points_t pts,
                                     const uint8_t* usable, int th, int32_t* kf_match, int* n_matches) {
    View K(*KFv);
    std::vector<char> taken(kf_taken, kf_taken + KFv->n);
    for (int j = 0; j < KFv->n; ++j) kf_match[j] = -1;
    int nmatches = 0;
    for (int iMP = 0; iMP < pts.n; iMP++) {
        if (!usable[iMP]) continue;
        int bestDist = INT_MAX;
        const int bestIdx = kf_project_best(K, row3(pts.pos, iMP), row3(pts.normal, iMP), pts.dmin[iMP],
                                            pts.dmax[iMP], pts.desc + (size_t)iMP * 32, (float)th, false, &taken,
                                            &bestDist);
        if (bestIdx < 0 && bestDist == INT_MAX) continue;
        if (bestDist <= TH_LOW) {
            taken[bestIdx] = 1;
            kf_match[bestIdx] = iMP;
            nmatches++;
        }
    }
    *n_matches = nmatches;
    return ORB_OK;
}

int oracle_fuse(const orb_frame_view_t* KFv, orb_map_points_t pts, const uint8_t* usable, float th, int scw,
                int32_t* best_idx, int* n_fused) {
    View K(*KFv);
    int nFused = 0;
    for (int i = 0; i < pts.n; i++) {
        best_idx[i] = -1;
        if (!usable[i]) continue;
        int bestDist = INT_MAX;
        const int bestIdx = kf_project_best(K, row3(pts.pos, i), row3(pts.normal, i), pts.dmin[i], pts.dmax[i],
                                            pts.desc + (size_t)i * 32, th, scw != 0, nullptr, &bestDist);
        if (bestIdx >= 0 && bestDist <= TH_LOW) {
            best_idx[i] = bestIdx;
            nFused++;
        }
    }
    *n_fused = nFused;
    return ORB_OK;
}

// SearchBySim3 (ORBmatcher.cc:1267-1505): one direction (p3Dc_other = sR * (Rw p + tw) + t).
static void sim3_direction(const orb_frame_view_t& src, orb_map_points_t mp, const uint8_t* usable,
                           const View& dst, const float* sR, const float* t, float th, std::vector<int>& vnMatch) {
    const float fx = src.fx, fy = src.fy, cx = src.cx, cy = src.cy;  // pKF1's calibration (1270-1273)
    for (int i1 = 0; i1 < src.n; i1++) {
        if (!usable[i1]) continue;
        const float* p3Dw = row3(mp.pos, i1);
        float p3Dc1[3], p3Dc2[3];
        ocv::gemm3_add(src.Rcw, p3Dw, src.tcw, p3Dc1);
        ocv::gemm3_add(sR, p3Dc1, t, p3Dc2);
        if (p3Dc2[2] < 0.0) continue;
        float invz = 1.0 / p3Dc2[2];
        float x = p3Dc2[0] * invz;
        float y = p3Dc2[1] * invz;
        float u = std::fma(fx, x, cx);
        float v = std::fma(fy, y, cy);
        if (!dst.in_image(u, v)) continue;
        float maxDistance = mp.dmax[i1];
        float minDistance = mp.dmin[i1];
        float dist3D = ocv::norm3(p3Dc2);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        float ratio = dist3D / minDistance;
        const int nPredictedLevel = dst.predict_level(ratio);
        float radius = th * dst.v.scale_factors[nPredictedLevel];
        std::vector<size_t> vIndices = dst.kf_area(u, v, radius);
        if (vIndices.empty()) continue;
        const uint8_t* dMP = mp.desc + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestIdx = -1;
        for (size_t idx : vIndices) {
            const orb_keypoint_t& kp = dst.v.kps[idx];
            if (kp.octave < nPredictedLevel - 1 || kp.octave > nPredictedLevel) continue;
            int dist = dist256(dMP, dst.desc(idx));
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_HIGH) vnMatch[i1] = bestIdx;
    }
}

int oracle_search_by_sim3(const orb_frame_view_t* KF1, orb_map_points_t mp1, const uint8_t* usable1,
                          const orb_frame_view_t* KF2, orb_map_points_t mp2, const uint8_t* usable2, const float* sR12,
                          const float* t12, const float* sR21, const float* t21, float th, int32_t* match12,
                          int* n_found) {
    View V1(*KF1), V2(*KF2);
    std::vector<int> vnMatch1(KF1->n, -1), vnMatch2(KF2->n, -1);
    // KF1 -> KF2 uses pKF1's calibration for the projection into KF2 (1270-1273, 1338-1339)
    sim3_direction(*KF1, mp1, usable1, V2, sR21, t21, th, vnMatch1);
    // KF2 -> KF1, again with pKF1's fx..cy
    orb_frame_view_t src2 = *KF2;
    src2.fx = KF1->fx;
    src2.fy = KF1->fy;
    src2.cx = KF1->cx;
    src2.cy = KF1->cy;
    sim3_direction(src2, mp2, usable2, V1, sR12, t12, th, vnMatch2);
    int nFound = 0;
    for (int i1 = 0; i1 < KF1->n; i1++) {
        match12[i1] = -1;
        int idx2 = vnMatch1[i1];
        if (idx2 >= 0) {
            int idx1 = vnMatch2[idx2];
            if (idx1 == i1) {
                match12[i1] = idx2;
                nFound++;
            }
        }
    }
    *n_found = nFound;
    return ORB_OK;
}

// CheckDistEpipolarLine (ORBmatcher.cc:136-153)
static bool check_dist_epipolar_line(const orb_keypoint_t& kp1, const orb_keypoint_t& kp2, const float* F12,
                                     const orb_frame_view_t& KF2) {
    // g++ -O3 -march=native contraction of the reference's expressions (scripts/contraction_check.sh)
    const float a = std::fma(kp1.x, F12[0], kp1.y * F12[3]) + F12[6];
    const float b = std::fma(kp1.x, F12[1], kp1.y * F12[4]) + F12[7];
    const float c = std::fma(kp1.y, F12[5], kp1.x * F12[2]) + F12[8];
    const float num = std::fma(b, kp2.y, a * kp2.x) + c;
    const float den = std::fma(a, a, b * b);
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * KF2.level_sigma2[kp2.octave];
}

int oracle_search_for_triangulation(const orb_frame_view_t* KF1, const uint8_t* has_mp1, orb_feature_vector_t fv1,
                                    const orb_frame_view_t* KF2, const uint8_t* has_mp2, orb_feature_vector_t fv2,
                                    const float* F12, float nnratio, int check_ori, int32_t* match12,
                                    int* n_matches) {
    (void)nnratio;
    int nmatches = 0;
    std::vector<char> vbMatched2(KF2->n, 0);
    for (int i = 0; i < KF1->n; ++i) match12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    fv_walk(fv1, fv2, [&](int a, int b) {
        for (int i1 = fv1.offsets[a]; i1 < fv1.offsets[a + 1]; i1++) {
            const int idx1 = fv1.features[i1];
            if (has_mp1[idx1]) continue;
            const orb_keypoint_t& kp1 = KF1->kps[idx1];
            const uint8_t* d1 = KF1->desc + (size_t)idx1 * 32;
            std::vector<std::pair<int, size_t>> vDistIndex;
            for (int i2 = fv2.offsets[b]; i2 < fv2.offsets[b + 1]; i2++) {
                const size_t idx2 = fv2.features[i2];
                if (vbMatched2[idx2] || has_mp2[idx2]) continue;
                const int dist = dist256(d1, KF2->desc + idx2 * 32);
                if (dist > TH_LOW) continue;
                vDistIndex.push_back(std::make_pair(dist, idx2));
            }
            if (vDistIndex.empty()) continue;
            std::sort(vDistIndex.begin(), vDistIndex.end());
            int BestDist = vDistIndex.front().first;
            int DistTh = round(2 * BestDist);
            for (size_t id = 0; id < vDistIndex.size(); id++) {
                if (vDistIndex[id].first > DistTh) break;
                int currentIdx2 = vDistIndex[id].second;
                const orb_keypoint_t& kp2 = KF2->kps[currentIdx2];
                if (check_dist_epipolar_line(kp1, kp2, F12, *KF2)) {
                    vbMatched2[currentIdx2] = 1;
                    match12[idx1] = currentIdx2;
                    nmatches++;
                    if (check_ori) {
                        float rot = kp1.angle - kp2.angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = round(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        rotHist[bin].push_back(idx1);
                    }
                    break;
                }
            }
        }
    });
    if (check_ori) rot_filter(rotHist, match12, nmatches);
    *n_matches = nmatches;
    return ORB_OK;
}

}  // extern "C"
