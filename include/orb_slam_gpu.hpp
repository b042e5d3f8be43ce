// orb_slam_gpu.hpp — header-only C++ facade re-exposing the reference's class API
// (ORB_SLAM::ORBextractor, include/ORBextractor.h:30-80; ORB_SLAM::ORBmatcher,
// include/ORBmatcher.h:36-108) on top of the C ABI in orb_abi.h (liborb_hip.so).
//
// Tracking / LocalMapping keep calling
//     (*mpORBextractor)(im, cv::Mat(), mvKeys, mDescriptors);                 // Frame.cc:60
//     ORBmatcher(0.9, true).SearchForInitialization(F1, F2, prev, m12, 100);  // Tracking.cc:392-393
// unchanged once Frame.cc / Tracking.cc include this header instead of ORBextractor.h and
// ORBmatcher.h and alias the classes.  With ORB_WITH_OPENCV defined the
// cv::InputArray / cv::KeyPoint overloads are available; without OpenCV the POD overloads
// are (std::vector<orb_keypoint_t>, row-major N x 32 descriptor bytes).
//
// Error behaviour: the reference asserts on bad input (ORBextractor.cc:725) and has no
// status codes; the facade throws std::runtime_error carrying orb_last_error() for any
// non-OK status, and keeps the reference's early return on an empty image
// (ORBextractor.cc:721-722: outputs untouched).
#ifndef ORB_SLAM_GPU_HPP
#define ORB_SLAM_GPU_HPP

#include <climits>
#include <cstdint>
#include <stdexcept>
#include <utility>
#include <string>
#include <vector>

#include "orb_abi.h"

#ifdef ORB_WITH_OPENCV
#include <opencv2/core/core.hpp>
#endif

namespace ORB_SLAM {
namespace gpu {

inline void orb_check(int st) {
    if (st < 0) throw std::runtime_error(std::string("orb: ") + orb_last_error() + " (status " + std::to_string(st) + ")");
}

class ORBextractor {
public:
    enum { HARRIS_SCORE = ORB_HARRIS_SCORE, FAST_SCORE = ORB_FAST_SCORE };

    ORBextractor(int nfeatures = 1000, float scaleFactor = 1.2f, int nlevels = 8, int scoreType = FAST_SCORE,
                 int fastTh = 20, int device = 0, int maxBatch = 1)
        : nlevels_(nlevels), scaleFactor_(scaleFactor) {
        orb_check(orb_extractor_create(nfeatures, scaleFactor, nlevels, scoreType, fastTh, device, maxBatch, &h_));
        cap_ = orb_get_max_keypoints(h_);
    }
    ~ORBextractor() { orb_extractor_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // ORBextractor::operator() on a POD image (u8, w x h, row pitch `stride`).
    void operator()(const uint8_t* img, int w, int h, int stride, std::vector<orb_keypoint_t>& keypoints,
                    std::vector<uint8_t>& descriptors) {
        if (w <= 0 || h <= 0) return;  // _image.empty(): outputs untouched
        keypoints.resize(cap_);
        descriptors.resize((size_t)cap_ * 32);
        int n = 0;
        orb_check(orb_extract(h_, img, w, h, stride, keypoints.data(), cap_, descriptors.data(), &n));
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);  // n == 0: the reference's _descriptors.release()
    }

#ifdef ORB_WITH_OPENCV
    // The reference signature (ORBextractor.h:43-45).  The mask is ignored, as by the
    // reference's FAST (ORBextractor.cc:601-607).
    void operator()(cv::InputArray _image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint>& _keypoints,
                    cv::OutputArray _descriptors) {
        if (_image.empty()) return;
        cv::Mat image = _image.getMat();
        CV_Assert(image.type() == CV_8UC1);
        std::vector<orb_keypoint_t> k;
        std::vector<uint8_t> d;
        (*this)(image.data, image.cols, image.rows, (int)image.step, k, d);
        _keypoints.clear();
        _keypoints.reserve(k.size());
        for (const orb_keypoint_t& p : k)
            _keypoints.push_back(cv::KeyPoint(p.x, p.y, p.size, p.angle, p.response, p.octave, p.class_id));
        if (k.empty()) {
            _descriptors.release();
        } else {
            _descriptors.create((int)k.size(), 32, CV_8U);
            cv::Mat D = _descriptors.getMat();
            for (size_t i = 0; i < k.size(); ++i) std::copy(&d[i * 32], &d[i * 32] + 32, D.ptr<uint8_t>((int)i));
        }
    }
#endif

    int inline GetLevels() { return nlevels_; }
    float inline GetScaleFactor() { return scaleFactor_; }
    orb_extractor_t* handle() { return h_; }

private:
    orb_extractor_t* h_ = nullptr;
    int nlevels_;
    float scaleFactor_;
    int cap_ = 0;
};

// The matcher-facing part of ORB_SLAM::Frame (Frame.h:43-138) for the POD overloads.
struct FrameView {
    const orb_keypoint_t* keysUn;  // mvKeysUn
    const uint8_t* descriptors;    // mDescriptors, N x 32
    int N;
    orb_frame_bounds_t bounds;     // mnMinX, mnMaxX, mnMinY, mnMaxY (static, first frame)
};

class ORBmatcher {
public:
    static const int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;  // ORBmatcher.cc:40-42

    ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orb_descriptor_distance(a, b); }

    // SearchForInitialization (ORBmatcher.cc:598-713): vbPrevMatched is N1 x {x, y}.
    int SearchForInitialization(const FrameView& F1, const FrameView& F2, std::vector<float>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10) {
        vnMatches12.assign(F1.N, -1);
        int n = 0;
        orb_check(orb_search_for_initialization(F1.keysUn, F1.descriptors, F1.N, F2.keysUn, F2.descriptors, F2.N,
                                                F1.bounds, mfNNratio, mbCheckOrientation ? 1 : 0, windowSize,
                                                vbPrevMatched.data(), vnMatches12.data(), &n));
        return n;
    }

    // ---- the rest of the family over POD views (orb_abi.h documents every flag array).
    // Outputs are indices: the caller maps them back to MapPoint* exactly where the
    // reference assigns (vpMapPointMatches[j] = pMP ...).

    // SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (ORBmatcher.cc:155-284):
    // vpMapPointMatches[j] = KF keypoint index whose MapPoint matched F keypoint j, or -1.
    int SearchByBoW(const orb_frame_view_t& KF, const uint8_t* kfUsable, const orb_feature_vector_t& kfFV,
                    const orb_frame_view_t& F, const orb_feature_vector_t& fFV, std::vector<int>& vpMapPointMatches,
                    int device = 0) {
        vpMapPointMatches.assign(F.n, -1);
        int n = 0;
        orb_check(orb_search_by_bow_kf_f(&KF, kfUsable, kfFV, &F, fFV, mfNNratio, mbCheckOrientation, vpMapPointMatches.data(), &n, device));
        return n;
    }
    // SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12) (ORBmatcher.cc:715-850).
    int SearchByBoW(const orb_frame_view_t& KF1, const uint8_t* usable1, const orb_feature_vector_t& fv1,
                    const orb_frame_view_t& KF2, const uint8_t* usable2, const orb_feature_vector_t& fv2,
                    std::vector<int>& vpMatches12, int device = 0) {
        vpMatches12.assign(KF1.n, -1);
        int n = 0;
        orb_check(orb_search_by_bow_kf_kf(&KF1, usable1, fv1, &KF2, usable2, fv2, mfNNratio, mbCheckOrientation, vpMatches12.data(), &n, device));
        return n;
    }
    // SearchForTriangulation (ORBmatcher.cc:852-1014): vMatchedPairs (i1, i2) ascending in i1.
    int SearchForTriangulation(const orb_frame_view_t& KF1, const uint8_t* hasMP1, const orb_feature_vector_t& fv1,
                               const orb_frame_view_t& KF2, const uint8_t* hasMP2, const orb_feature_vector_t& fv2,
                               const float F12[9], std::vector<std::pair<size_t, size_t> >& vMatchedPairs,
                               int device = 0) {
        std::vector<int> m12(KF1.n, -1);
        int n = 0;
        orb_check(orb_search_for_triangulation(&KF1, hasMP1, fv1, &KF2, hasMP2, fv2, F12, mfNNratio, mbCheckOrientation, m12.data(), &n, device));
        vMatchedPairs.clear();
        for (int i = 0; i < KF1.n; ++i)
            if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
        return n;
    }
    // WindowSearch (ORBmatcher.cc:409-516): vpMapPointMatches2[i2] = F1 index or -1.
    int WindowSearch(const orb_frame_view_t& F1, const uint8_t* usable1, const orb_frame_view_t& F2, int windowSize,
                     std::vector<int>& vpMapPointMatches2, int minScaleLevel = 0, int maxScaleLevel = INT_MAX,
                     int device = 0) {
        vpMapPointMatches2.assign(F2.n, -1);
        int n = 0;
        orb_check(orb_window_search(&F1, usable1, &F2, windowSize, minScaleLevel, maxScaleLevel, mfNNratio, mbCheckOrientation, vpMapPointMatches2.data(), &n, device));
        return n;
    }
    // SearchByProjection(Frame& F, vector<MapPoint*>, th) (ORBmatcher.cc:49-125) over the
    // isInFrustum fields; newMatches[j] = MapPoint row assigned to F keypoint j, or -1.
    int SearchByProjection(const orb_frame_view_t& F, const uint8_t* fTaken, int nMP, const uint8_t* usable,
                           const float* projX, const float* projY, const int32_t* level, const float* viewCos,
                           const uint8_t* mpDesc, float th, std::vector<int>& newMatches, int device = 0) {
        newMatches.assign(F.n, -1);
        int n = 0;
        orb_check(orb_search_by_projection_local(&F, fTaken, nMP, usable, projX, projY, level, viewCos, mpDesc, th, mfNNratio, newMatches.data(), &n, device));
        return n;
    }
    // SearchByProjection(Frame& F1, Frame& F2, windowSize, vpMapPointMatches2) (519-594).
    int SearchByProjection(const orb_frame_view_t& F1, const orb_map_points_t& mp1, const uint8_t* usable1,
                           const orb_frame_view_t& F2, const uint8_t* f2Taken, int windowSize,
                           std::vector<int>& newMatches2, int device = 0) {
        newMatches2.assign(F2.n, -1);
        int n = 0;
        orb_check(orb_search_by_projection_f2f(&F1, mp1, usable1, &F2, f2Taken, windowSize, mfNNratio, newMatches2.data(), &n, device));
        return n;
    }
    // SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th) (1507-1620).
    int SearchByProjection(const orb_frame_view_t& Cur, const uint8_t* curTaken, const orb_frame_view_t& Last,
                           const orb_map_points_t& mp, const uint8_t* usable, float th, std::vector<int>& newMatches,
                           int device = 0) {
        newMatches.assign(Cur.n, -1);
        int n = 0;
        orb_check(orb_search_by_projection_motion(&Cur, curTaken, &Last, mp, usable, th, mbCheckOrientation, newMatches.data(), &n, device));
        return n;
    }
    // SearchByProjection(Frame& CurrentFrame, KeyFrame*, sAlreadyFound, th, ORBdist) (1622-1746).
    int SearchByProjection(const orb_frame_view_t& Cur, const uint8_t* curTaken, const orb_frame_view_t& KF,
                           const orb_map_points_t& mp, const uint8_t* usable, float th, int ORBdist,
                           std::vector<int>& newMatches, int device = 0) {
        newMatches.assign(Cur.n, -1);
        int n = 0;
        orb_check(orb_search_by_projection_reloc(&Cur, curTaken, &KF, mp, usable, th, ORBdist, mbCheckOrientation, newMatches.data(), &n, device));
        return n;
    }
    // SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (286-407); KF's pose = Scw's.
    int SearchByProjection(const orb_frame_view_t& KFscw, const uint8_t* kfTaken, const orb_map_points_t& pts,
                           const uint8_t* usable, int th, std::vector<int>& newMatches, int device = 0) {
        newMatches.assign(KFscw.n, -1);
        int n = 0;
        orb_check(orb_search_by_projection_sim3(&KFscw, kfTaken, pts, usable, th, newMatches.data(), &n, device));
        return n;
    }
    // SearchBySim3 (ORBmatcher.cc:1267-1505): vpMatches12[i1] = agreeing KF2 index or -1.
    int SearchBySim3(const orb_frame_view_t& KF1, const orb_map_points_t& mp1, const uint8_t* usable1,
                     const orb_frame_view_t& KF2, const orb_map_points_t& mp2, const uint8_t* usable2,
                     const float sR12[9], const float t12[3], const float sR21[9], const float t21[3], float th,
                     std::vector<int>& vpMatches12, int device = 0) {
        vpMatches12.assign(KF1.n, -1);
        int n = 0;
        orb_check(orb_search_by_sim3(&KF1, mp1, usable1, &KF2, mp2, usable2, sR12, t12, sR21, t21, th, vpMatches12.data(), &n, device));
        return n;
    }
    // Fuse(KeyFrame*, vector<MapPoint*>, th) / Fuse(KeyFrame*, Scw, ..., th) (1016-1265):
    // bestIdx[i] = KF keypoint point i fuses with, or -1; the caller applies Replace /
    // AddObservation in point order.
    int Fuse(const orb_frame_view_t& KF, const orb_map_points_t& pts, const uint8_t* usable, float th, bool scw,
             std::vector<int>& bestIdx, int device = 0) {
        bestIdx.assign(pts.n, -1);
        int n = 0;
        orb_check(orb_fuse(&KF, pts, usable, th, scw ? 1 : 0, bestIdx.data(), &n, device));
        return n;
    }

#ifdef ORB_WITH_OPENCV
    static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
        return orb_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
    }
#endif

private:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace gpu
}  // namespace ORB_SLAM

#endif
