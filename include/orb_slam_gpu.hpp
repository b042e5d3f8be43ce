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

#include <cstdint>
#include <stdexcept>
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
