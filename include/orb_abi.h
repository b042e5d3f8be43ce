/*
 * orb_abi.h — C ABI of the MI355X-native ORB front end (liborb_hip.so).
 *
 * Drop-in boundary for the reference's per-frame feature front end:
 *   ORB_SLAM::ORBextractor (reference include/ORBextractor.h:30-80, src/ORBextractor.cc:457-822)
 *   ORB_SLAM::ORBmatcher   (reference include/ORBmatcher.h:36-108, src/ORBmatcher.cc)
 * Plain pointers and sizes only; no C++ types, no exceptions across the boundary.
 * Every entry point returns an int status: ORB_OK (0) or a negative errno-style code.
 *
 * Threading mirrors the reference: an extractor handle owns one HIP stream plus its
 * device workspace and is used by one host thread at a time (the reference extractor is
 * stateful, ORBextractor.h:74-75).  Distinct handles may run concurrently, on the same
 * or on different devices.
 */
#ifndef ORB_ABI_H
#define ORB_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define ORB_OK 0
#define ORB_EINVAL (-22)   /* bad argument / unsupported configuration                  */
#define ORB_ENOMEM (-12)   /* device or host allocation failed                          */
#define ORB_ERANGE (-34)   /* output capacity too small                                 */
#define ORB_EDEVICE (-5)   /* HIP runtime error (message via orb_last_error)           */
#define ORB_ENOTSUP (-95)  /* configuration the reference itself cannot run            */

/* ---- score types (reference ORBextractor.h:36) ------------------------------------- */
#define ORB_HARRIS_SCORE 0
#define ORB_FAST_SCORE 1

/* Keypoint record, layout-identical to cv::KeyPoint (OpenCV 2.4, 28 bytes) and to the
 * on-disk record of reference include/SaveLoadWorld.h:1406-1425. */
typedef struct orb_keypoint {
    float x, y;        /* pt, image (level-0) pixel coordinates                       */
    float size;        /* (int)(31 * scaleFactor^octave)                              */
    float angle;       /* degrees in [0, 360], IC_Angle via fastAtan2                 */
    float response;    /* FAST score (or Harris response)                             */
    int32_t octave;    /* pyramid level                                               */
    int32_t class_id;  /* always -1                                                   */
} orb_keypoint_t;

typedef struct orb_extractor orb_extractor_t; /* opaque handle */

/* Last error message of the calling thread (never NULL). */
const char* orb_last_error(void);

/* Library build identifier, e.g. "orb_hip gfx950 <date>". */
const char* orb_version(void);

/* ---- ORBextractor ------------------------------------------------------------------ */
/* Replaces ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels, scoreType, fastTh)
 * (reference ORBextractor.h:38, ORBextractor.cc:457-511).  `device` is the HIP ordinal;
 * `max_batch` sizes the device workspace for orb_extract_batch_device (>= 1). */
int orb_extractor_create(int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th,
                         int device, int max_batch, orb_extractor_t** out);
int orb_extractor_destroy(orb_extractor_t* h);

/* ORBextractor::GetLevels / GetScaleFactor (reference ORBextractor.h:47-51). */
int orb_get_levels(const orb_extractor_t* h);
float orb_get_scale_factor(const orb_extractor_t* h);
/* Per-frame keypoint capacity of the batched entry points: sum of the per-level quotas
 * (== nfeatures for every configuration whose rounded quotas do not overshoot). */
int orb_get_max_keypoints(const orb_extractor_t* h);
/* Per-level quotas (mnFeaturesPerLevel, ORBextractor.cc:476-487) and scale factors
 * (mvScaleFactor, ORBextractor.cc:462-465); arrays of length orb_get_levels(). */
int orb_get_level_info(const orb_extractor_t* h, int* features_per_level, float* scale_factors);

/* ORBextractor::operator()(image, mask=cv::Mat(), keypoints, descriptors)
 * (reference ORBextractor.cc:718-779) on ONE host image.
 *   img: u8 grayscale, w x h, row pitch `stride` bytes (continuous or strided, CV_8UC1).
 *   kps_out: capacity `kps_cap` records; desc_out: capacity kps_cap x 32 bytes (row-major).
 *   *n_out: number of keypoints written (<= nfeatures).  Order = the reference's order:
 *   level-major, cells row-major, libstdc++ nth_element permutation inside retainBest.
 * An empty image (w == 0 or h == 0) returns ORB_OK with *n_out = 0 and touches nothing,
 * like the reference's early return (ORBextractor.cc:721-722).  The mask is ignored by the
 * reference's FAST (ORBextractor.cc:601-607) and is not part of this ABI. */
int orb_extract(orb_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, orb_keypoint_t* kps_out,
                int kps_cap, uint8_t* desc_out, int* n_out);

/* Batched extraction on device-resident frames (the GPU-native entry point).
 *   d_imgs: B frames, frame k at d_imgs + k*frame_pitch, each w x h at row pitch `stride`.
 *   d_kps: B x cap records, cap = orb_get_max_keypoints(h) (frame k at d_kps + k*cap);
 *   d_desc: B x cap x 32 bytes; d_counts: B int32 keypoint counts.
 *   stream: hipStream_t to enqueue on (NULL = the null stream, as in every HIP API; the
 *   handle's own stream serves only the host-buffer entry points).  Asynchronous: returns
 *   after enqueueing; work on other streams must be ordered against it by the caller
 *   (events), and the stream synchronised before reading outputs. */
int orb_extract_batch_device(orb_extractor_t* h, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                             int64_t frame_pitch, orb_keypoint_t* d_kps, uint8_t* d_desc, int32_t* d_counts,
                             void* stream);

/* Host-buffer batch: copies B host frames in, runs, copies results out (synchronous).
 * kps_out / desc_out / n_out laid out as for the device variant. */
int orb_extract_batch(orb_extractor_t* h, int B, const uint8_t* imgs, int w, int hgt, int stride,
                      int64_t frame_pitch, orb_keypoint_t* kps_out, uint8_t* desc_out, int32_t* n_out);

/* Colour frames: Tracking::GrabImage's cvtColor(image, im, mbRGB ? CV_RGB2GRAY : CV_BGR2GRAY)
 * (reference Tracking.cc:202-207; OpenCV 2.4 fixed-point luma, exact) fused into the level-0
 * pass, then the same extraction.  channels 3 or 4 (interleaved u8, row pitch `stride` bytes >=
 * w * channels); rgb != 0 for RGB channel order, 0 for BGR.  Otherwise as orb_extract_batch_device
 * / orb_extract. */
int orb_extract_batch_device_color(orb_extractor_t* h, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                                   int64_t frame_pitch, int channels, int rgb, orb_keypoint_t* d_kps, uint8_t* d_desc,
                                   int32_t* d_counts, void* stream);
int orb_extract_color(orb_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, int channels, int rgb,
                      orb_keypoint_t* kps_out, int kps_cap, uint8_t* desc_out, int* n_out);

/* ---- ORBmatcher -------------------------------------------------------------------- */
/* ORBmatcher::DescriptorDistance (reference ORBmatcher.cc:1794-1810; DBoW2 FORB.cpp:81-101). */
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Frame geometry needed by Frame::GetFeaturesInArea / PosInGrid (reference Frame.cc:73-86,
 * 200-277): image bounds (mnMinX..mnMaxY, from the first frame) of the 64 x 48 grid. */
typedef struct orb_frame_bounds {
    int min_x, max_x, min_y, max_y;
} orb_frame_bounds_t;

/* ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12,
 * windowSize) (reference ORBmatcher.cc:598-713) for ONE frame pair, host buffers.
 *   kps1/desc1 (n1), kps2/desc2 (n2): the frames' mvKeysUn and mDescriptors.
 *   prev_xy: n1 x 2 floats, vbPrevMatched, updated in place (ORBmatcher.cc:707-710).
 *   matches12: n1 ints, vnMatches12 (-1 = unmatched).  Returns nmatches in *n_matches. */
int orb_search_for_initialization(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1,
                                  const orb_keypoint_t* kps2, const uint8_t* desc2, int n2,
                                  orb_frame_bounds_t bounds, float nnratio, int check_ori, int window,
                                  float* prev_xy, int32_t* matches12, int* n_matches);

/* Batched SearchForInitialization on device-resident extractor output.
 * Pair p matches frame pair_f1[p] against frame pair_f2[p] of a batch laid out as by
 * orb_extract_batch_device (d_kps / d_desc / d_counts with per-frame capacity `cap`).
 *   d_prev_xy: P x cap x 2 floats (in/out); NULL means "vbPrevMatched = F1 keypoints"
 *              (Tracking::FirstInitialization, reference Tracking.cc:366-368) and no update.
 *   d_matches12: P x cap int32; d_nmatches: P int32.  d_desc 16-B aligned.  Asynchronous on
 *   `stream`.
 * cap <= 8192.  One workgroup per pair holds up to nmax octave-0 keypoints per frame in LDS:
 * nmax = min(cap, 1024) for P < 256 pairs, min(cap, 1024, max(256, ~9/40 cap)) otherwise (the
 * extractor keeps at most 0.217 nFeatures at level 0).  A pair over nmax (another producer, the
 * reference init extractor's nFeatures*2 at 1280x720) is redone exactly by the same workgroup
 * with its staged arrays in a grow-only scratch kept per (device, stream); every pair is exact
 * and there is one launch per call. */
int orb_search_for_initialization_batch_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                               const int32_t* d_counts, int cap, int P, const int32_t* d_pair_f1,
                                               const int32_t* d_pair_f2, orb_frame_bounds_t bounds, float nnratio,
                                               int check_ori, int window, float* d_prev_xy, int32_t* d_matches12,
                                               int32_t* d_nmatches, void* stream);
/* Release the large-capacity scratch kept for `stream` on the current device (freed in stream
 * order, after the launches already queued on it).  Call before destroying a stream that ran
 * orb_search_for_initialization_batch_device; a later call on the stream re-creates it.  No
 * reference counterpart (resource hook of the batched entry point). */
int orb_match_release_stream_scratch(void* stream);
/* A HIP stream on the current device with a hardware queue of its own, for callers that
 * overlap H2D copies, extraction and D2H copies on separate streams (the host-fed step of
 * ORBextractor::operator() callers, bench.py host_fed).  Plain streams share the runtime's
 * GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin, so a copy stream can land on
 * the queue of an extraction stream and serialise behind it; this stream is created with a CU
 * mask naming every CU of the device (hipExtStreamCreateWithCUMask), which the runtime serves
 * from a queue of its own whatever GPU_MAX_HW_QUEUES says.  Non-blocking w.r.t. the null stream
 * is NOT implied (order it with events).  orb_stream_destroy releases it (and the matcher scratch
 * kept for it).  No reference counterpart (resource hook). */
int orb_stream_create_dedicated(void** out_stream);
int orb_stream_destroy(void* stream);

/* ---- the rest of the ORBmatcher family (GPU: csrc/orb_match.hip) ------------------- */
/* All entry points below take HOST buffers, run on the device of `device`, and are
 * synchronous.  Map state the reference reads through MapPoint / KeyFrame methods
 * (isBad, IsInKeyFrame, "already found" sets, outlier flags) arrives as caller-evaluated
 * per-element `usable` / `taken` flags; each entry point names the reference condition its
 * flags encode.  Results are indices (the caller maps them back to MapPoint*), so no map
 * object crosses the boundary.  Pose-level cv::Mat algebra the reference performs once per
 * call (Scw decomposition, Sim3 composition, -R^T t) is done by the caller with the
 * reference's own expressions and passed in; the per-point geometry runs on the device. */

#define ORB_MAX_VIEW_LEVELS 16

/* A Frame or KeyFrame as the matchers see it (reference Frame.h:43-138, KeyFrame.h). */
typedef struct orb_frame_view {
    const orb_keypoint_t* kps;  /* mvKeysUn, n records                                   */
    const uint8_t* desc;        /* mDescriptors, n x 32 bytes row-major                  */
    int32_t n;
    int32_t nlevels;            /* mnScaleLevels (<= ORB_MAX_VIEW_LEVELS)                */
    orb_frame_bounds_t bounds;  /* mnMinX .. mnMaxY; grid = 64 x 48 cells over them       */
    float scale_factors[ORB_MAX_VIEW_LEVELS]; /* mvScaleFactors (Frame.cc:95-103)        */
    float level_sigma2[ORB_MAX_VIEW_LEVELS];  /* mvLevelSigma2                           */
    float fx, fy, cx, cy;       /* calibration                                            */
    float Rcw[9];               /* rotation world->camera, row-major (mRcw / GetRotation) */
    float tcw[3];               /* translation (mtcw / GetTranslation)                    */
    float Ow[3];                /* camera centre (mOw / GetCameraCenter)                  */
} orb_frame_view_t;

/* MapPoint attributes read by the projection matchers (reference MapPoint.h). */
typedef struct orb_map_points {
    const float* pos;     /* n x 3 GetWorldPos                                            */
    const float* normal;  /* n x 3 GetNormal (NULL where unused)                          */
    const float* dmin;    /* n GetMinDistanceInvariance (NULL where unused)               */
    const float* dmax;    /* n GetMaxDistanceInvariance (NULL where unused)               */
    const uint8_t* desc;  /* n x 32 GetDescriptor (NULL where the frame's row is used)    */
    int32_t n;
} orb_map_points_t;

/* DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>, FeatureVector.h:21-49) as CSR:
 * ascending node ids nodes[n_nodes], offsets[n_nodes + 1], feature indices features[]. */
typedef struct orb_feature_vector {
    const uint32_t* nodes;
    const int32_t* offsets;
    const int32_t* features;
    int32_t n_nodes;
} orb_feature_vector_t;

/* Frame::GetFeaturesInArea (Frame.cc:200-265) for q query windows (min/max level -1 = any),
 * or KeyFrame::GetFeaturesInArea (KeyFrame.cc:612-652, no level filter, `<= r`) when
 * keyframe != 0.  Output CSR: out_offsets[q + 1], out_indices[capacity]; ORB_ERANGE if the
 * candidates exceed `capacity` (out_offsets[q] then holds the required size). */
int orb_features_in_area(const orb_frame_view_t* view, int keyframe, int q, const float* x, const float* y,
                         const float* r, const int32_t* min_level, const int32_t* max_level, int32_t* out_offsets,
                         int32_t* out_indices, int capacity, int device);

/* Frame::isInFrustum (Frame.cc:137-198) for every MapPoint: in_view[i] (mbTrackInView),
 * proj_x/proj_y (mTrackProjX/Y), level (mnTrackScaleLevel), view_cos (mTrackViewCos).
 * mps.normal/dmin/dmax required. */
int orb_frame_is_in_frustum(const orb_frame_view_t* F, orb_map_points_t mps, float viewing_cos_limit,
                            uint8_t* in_view, float* proj_x, float* proj_y, int32_t* level, float* view_cos,
                            int device);

/* SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (ORBmatcher.cc:155-284).
 * kf_usable[i]: vpMapPointsKF[i] && !isBad().  f_match[j] = KF keypoint whose MapPoint is
 * matched to F keypoint j, or -1. */
int orb_search_by_bow_kf_f(const orb_frame_view_t* KF, const uint8_t* kf_usable, orb_feature_vector_t kf_fv,
                           const orb_frame_view_t* F, orb_feature_vector_t f_fv, float nnratio, int check_ori,
                           int32_t* f_match, int* n_matches, int device);

/* SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12) (ORBmatcher.cc:715-850).
 * usable1/usable2: vpMapPoints[i] && !isBad().  match12[i1] = idx2 or -1. */
int orb_search_by_bow_kf_kf(const orb_frame_view_t* KF1, const uint8_t* usable1, orb_feature_vector_t fv1,
                            const orb_frame_view_t* KF2, const uint8_t* usable2, orb_feature_vector_t fv2,
                            float nnratio, int check_ori, int32_t* match12, int* n_matches, int device);

/* SearchByBoW over many pairs per launch, on device-resident extractor output
 * (orb_extract_batch_device: d_kps / d_desc [B][cap], d_counts[B]) and the FeatureVectors of the
 * same frames (orb_vocabulary_transform_batch_device: d_fv_nodes [B][cap], d_fv_offsets
 * [B][cap + 1], d_fv_features [B][cap], d_fv_n [B]).  Pair p = frames (d_pair_a[p], d_pair_b[p]):
 *   kf_kf = 0: SearchByBoW(KeyFrame* = frame a, Frame& = frame b, vpMapPointMatches)
 *              (ORBmatcher.cc:155-284; Tracking.cc:927 with nnratio 0.7): d_match[p][j] = the
 *              frame-a keypoint matched to frame-b keypoint j, or -1;
 *   kf_kf = 1: SearchByBoW(KeyFrame* = a, KeyFrame* = b, vpMatches12) (ORBmatcher.cc:715-850;
 *              LoopClosing.cc:278 with 0.75): d_match[p][i1] = idx2 in frame b, or -1.
 * d_usable [B][cap]: the frame's keypoint has a MapPoint that is not bad (both sides for kf_kf =
 * 1, the KF side for kf_kf = 0); NULL = every keypoint.  d_match rows are written whole (-1 past
 * the count); d_nmatches[p] = the reference's return value.  cap <= 8192, d_desc 16-B aligned.
 * Asynchronous on `stream`. */
int orb_search_by_bow_batch_device(int kf_kf, const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                   const int32_t* d_counts, int cap, const uint32_t* d_fv_nodes,
                                   const int32_t* d_fv_offsets, const int32_t* d_fv_features, const int32_t* d_fv_n,
                                   int P, const int32_t* d_pair_a, const int32_t* d_pair_b, const uint8_t* d_usable,
                                   float nnratio, int check_ori, int32_t* d_match, int32_t* d_nmatches, void* stream);

/* SearchForTriangulation(KF1, KF2, F12, ...) (ORBmatcher.cc:852-1014) with
 * CheckDistEpipolarLine (136-153).  has_mp1/has_mp2: GetMapPointMatches()[i] != NULL.
 * F12 row-major 3x3.  match12[i1] = idx2 or -1 (vMatchedPairs = the i1 with match12 >= 0,
 * ascending). */
int orb_search_for_triangulation(const orb_frame_view_t* KF1, const uint8_t* has_mp1, orb_feature_vector_t fv1,
                                 const orb_frame_view_t* KF2, const uint8_t* has_mp2, orb_feature_vector_t fv2,
                                 const float* F12, float nnratio, int check_ori, int32_t* match12, int* n_matches,
                                 int device);

/* WindowSearch(F1, F2, windowSize, vpMapPointMatches2, minScaleLevel, maxScaleLevel)
 * (ORBmatcher.cc:409-516).  usable1[i1]: F1.mvpMapPoints[i1] && !isBad().
 * match21[i2] = i1 whose MapPoint lands on F2 keypoint i2, or -1. */
int orb_window_search(const orb_frame_view_t* F1, const uint8_t* usable1, const orb_frame_view_t* F2, int window,
                      int min_scale_level, int max_scale_level, float nnratio, int check_ori, int32_t* match21,
                      int* n_matches, int device);

/* SearchByProjection(Frame& F, vector<MapPoint*>, th) (ORBmatcher.cc:49-125) over MapPoints
 * already projected by Frame::isInFrustum.  usable[i]: mbTrackInView && !isBad();
 * f_taken[j]: F.mvpMapPoints[j] != NULL on entry.  f_match[j] = MapPoint index newly
 * assigned to F keypoint j, or -1. */
int orb_search_by_projection_local(const orb_frame_view_t* F, const uint8_t* f_taken, int n_mp, const uint8_t* usable,
                                   const float* proj_x, const float* proj_y, const int32_t* level,
                                   const float* view_cos, const uint8_t* mp_desc, float th, float nnratio,
                                   int32_t* f_match, int* n_matches, int device);

/* SearchByProjection(Frame& F1, Frame& F2, windowSize, vpMapPointMatches2)
 * (ORBmatcher.cc:519-594).  mp1.pos: F1's MapPoint positions (row i1); usable1[i1]:
 * pMP1 && !isBad() && not already in F2.mvpMapPoints; f2_taken[i2]: F2.mvpMapPoints[i2].
 * match2[i2] = i1 newly assigned, or -1. */
int orb_search_by_projection_f2f(const orb_frame_view_t* F1, orb_map_points_t mp1, const uint8_t* usable1,
                                 const orb_frame_view_t* F2, const uint8_t* f2_taken, int window, float nnratio,
                                 int32_t* match2, int* n_matches, int device);

/* SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th) (ORBmatcher.cc:
 * 1507-1620).  usable[i]: LastFrame.mvpMapPoints[i] && !mvbOutlier[i]; mp.pos row i.
 * cur_match[j] = LastFrame index newly assigned to Current keypoint j, or -1. */
int orb_search_by_projection_motion(const orb_frame_view_t* Cur, const uint8_t* cur_taken, const orb_frame_view_t* Last,
                                    orb_map_points_t mp, const uint8_t* usable, float th, int check_ori,
                                    int32_t* cur_match, int* n_matches, int device);

/* SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th, ORBdist)
 * (ORBmatcher.cc:1622-1746).  mp: the KF's MapPoints (pos, dmin, desc) row i; usable[i]:
 * pMP && !isBad() && !sAlreadyFound.count(pMP).  Cur->Ow = -Rcw^T tcw of the current pose. */
int orb_search_by_projection_reloc(const orb_frame_view_t* Cur, const uint8_t* cur_taken, const orb_frame_view_t* KF,
                                   orb_map_points_t mp, const uint8_t* usable, float th, int orb_dist,
                                   int check_ori, int32_t* cur_match, int* n_matches, int device);

/* SearchByProjection(KeyFrame* pKF, cv::Mat Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:
 * 286-407).  KF->Rcw/tcw/Ow = the Scw decomposition of 297-302; usable[i]: !isBad() &&
 * !spAlreadyFound.count(pMP); kf_taken[j]: vpMatched[j].  kf_match[j] = point index or -1. */
int orb_search_by_projection_sim3(const orb_frame_view_t* KF, const uint8_t* kf_taken, orb_map_points_t pts,
                                  const uint8_t* usable, int th, int32_t* kf_match, int* n_matches, int device);

/* SearchBySim3(KF1, KF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1267-1505).
 * mp1/mp2: the keyframes' MapPoints (pos, dmin, dmax, desc) by keypoint index; usable1/2:
 * pMP && !vbAlreadyMatched && !isBad().  sR12 = s12*R12, sR21 = (1/s12)*R12^T,
 * t21 = -sR21*t12 as the reference computes them (1288-1290).  match12[i1] = idx2 for the
 * mutually agreeing pairs, -1 elsewhere; *n_found = their count. */
int orb_search_by_sim3(const orb_frame_view_t* KF1, orb_map_points_t mp1, const uint8_t* usable1,
                       const orb_frame_view_t* KF2, orb_map_points_t mp2, const uint8_t* usable2, const float* sR12,
                       const float* t12, const float* sR21, const float* t21, float th, int32_t* match12,
                       int* n_found, int device);

/* Fuse(KeyFrame*, vector<MapPoint*>, th) (ORBmatcher.cc:1016-1134) when scw == 0, or
 * Fuse(KeyFrame*, cv::Mat Scw, vpPoints, th) (1136-1265) when scw != 0 (KF pose = the Scw
 * decomposition).  usable[i]: pMP && !isBad() && !IsInKeyFrame (resp. !spAlreadyFound).
 * best_idx[i] = KF keypoint the point fuses with (bestDist <= TH_LOW), or -1; the caller
 * applies Replace / AddObservation in point order (the map mutation stays on the host). */
int orb_fuse(const orb_frame_view_t* KF, orb_map_points_t pts, const uint8_t* usable, float th, int scw,
             int32_t* best_idx, int* n_fused, int device);

/* ---- Frame keypoint geometry (GPU: csrc/orb_frame.hip) ------------------------------ */
/* The camera as Tracking.cc:52-70 builds it: K4 = (fx, fy, cx, cy) of K = [fx 0 cx; 0 fy cy;
 * 0 0 1], dist4 = mDistCoef = (k1, k2, p1, p2).  cv::undistortPoints(pts, pts, K, mDistCoef,
 * noArray(), K) (OpenCV 2.4 cvUndistortPoints: double arithmetic, 5 fixed iterations) is
 * restated exactly on the device.  fx, fy must be finite and non-zero (ORB_EINVAL). */
/* Frame::UndistortKeyPoints (Frame.cc:289-319) over a [B][cap] extractor batch: slot i < counts[b]
 * of d_kps_un = that keypoint with pt undistorted, or copied unchanged when k1 == 0
 * (Frame.cc:291-295).  d_kps_un may equal d_kps.  Asynchronous on `stream`. */
int orb_undistort_keypoints_batch_device(const orb_keypoint_t* d_kps, const int32_t* d_counts, int cap, int B,
                                         const float* K4, const float* dist4, orb_keypoint_t* d_kps_un,
                                         void* stream);
/* The same for one frame's n keypoints in host buffers (synchronous; device -1 = current). */
int orb_undistort_keypoints(const orb_keypoint_t* kps, int n, const float* K4, const float* dist4, int device,
                            orb_keypoint_t* out);
/* cv::undistortPoints itself on n points xy[2n] -> out[2n] (no k1 == 0 shortcut). */
int orb_undistort_points(const float* xy, int n, const float* K4, const float* dist4, int device, float* out);
/* Frame::ComputeImageBounds (Frame.cc:321-349): the undistorted image corners' floor / ceil
 * when k1 != 0, else the image rectangle. */
int orb_compute_image_bounds(int cols, int rows, const float* K4, const float* dist4, int device,
                             orb_frame_bounds_t* out);

/* ---- the front end over a camera stream, overlapped (csrc/orb_pipeline.hip) ---------- */
/* B consecutive frames of one camera: ORBextractor::operator() on each (Frame::Frame,
 * Frame.cc:56-128) and SearchForInitialization(F_b, F_b+1) for b < B-1 with vbPrevMatched =
 * F_b's keypoints (Tracking.cc:366-368, 392-393).  The batch is cut into n_streams contiguous
 * chunks, each with its own extractor handle and HIP stream, so latency-bound kernels of
 * one chunk overlap the others; outputs equal the serial path's.  One handle = one caller. */
typedef struct orb_pipeline orb_pipeline_t; /* opaque handle */
int orb_pipeline_create(int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th, int device,
                        int max_batch, int n_streams, orb_pipeline_t** out);
int orb_pipeline_destroy(orb_pipeline_t* p);
int orb_pipeline_max_keypoints(const orb_pipeline_t* p);
int orb_pipeline_streams(const orb_pipeline_t* p);
/* Outputs as orb_extract_batch_device (d_kps/d_desc/d_counts, per-frame capacity
 * orb_pipeline_max_keypoints) and orb_search_for_initialization_batch_device (pair b = (b, b+1):
 * d_matches12 (B-1) x cap, d_nmatches B-1).  Ordered after earlier work on `stream` and
 * before later work on it (events); asynchronous. */
int orb_pipeline_extract_and_match(orb_pipeline_t* p, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                                   int64_t frame_pitch, orb_keypoint_t* d_kps, uint8_t* d_desc, int32_t* d_counts,
                                   orb_frame_bounds_t bounds, float nnratio, int check_ori, int window,
                                   int32_t* d_matches12, int32_t* d_nmatches, void* stream);
/* The same step for a calibrated camera with distortion (Frame::Frame: UndistortKeyPoints,
 * Frame.cc:69): after each chunk's extraction its keypoints are undistorted into d_kps_un
 * (orb_undistort_keypoints_batch_device; K4 / dist4 as there) and the pairs are matched on
 * mvKeysUn, with `bounds` = orb_compute_image_bounds of the camera.  K4 = NULL is
 * orb_pipeline_extract_and_match (d_kps_un unused). */
int orb_pipeline_extract_undistort_and_match(orb_pipeline_t* p, int B, const uint8_t* d_imgs, int w, int hgt,
                                             int stride, int64_t frame_pitch, const float* K4, const float* dist4,
                                             orb_keypoint_t* d_kps, orb_keypoint_t* d_kps_un, uint8_t* d_desc,
                                             int32_t* d_counts, orb_frame_bounds_t bounds, float nnratio,
                                             int check_ori, int window, int32_t* d_matches12, int32_t* d_nmatches,
                                             void* stream);
/* Per-stage HIP-event timing summed over the chunk handles (see orb_profile_*). */
int orb_pipeline_profile_enable(orb_pipeline_t* p, int enable);
int orb_pipeline_profile_read(orb_pipeline_t* p, double* stage_ms, int64_t* stage_launches, int nstages);

/* ---- MapPoint descriptor maintenance (GPU: csrc/orb_mappoint.hip) ------------------- */
/* MapPoint::ComputeDistinctiveDescriptors (reference src/MapPoint.cc:185-250) for M points:
 * point m's observed descriptors are rows offsets[m] .. offsets[m+1]-1 of desc (32 B each), in
 * the order of its std::map<KeyFrame*, size_t> observations; usable[r] = !pKF->isBad() for the
 * keyframe of row r (NULL = all).  best_row[m] = the row chosen as mDescriptor and
 * out_desc[m] = its bytes, or best_row[m] = -1 and out_desc[m] untouched when no row is usable
 * (the reference returns without changing mDescriptor).  <= 4000 rows per point.
 * Host buffers, synchronous. */
int orb_compute_distinctive_descriptors(int M, const int32_t* offsets, const uint8_t* desc, const uint8_t* usable,
                                        int32_t* best_row, uint8_t* out_desc, int device);
/* The same on device buffers (desc 16-B aligned); max_obs = the largest row count of a point.
 * Asynchronous on `stream`. */
int orb_compute_distinctive_descriptors_device(int M, const int32_t* d_offsets, const uint8_t* d_desc,
                                               const uint8_t* d_usable, int max_obs, int32_t* d_best_row,
                                               uint8_t* d_out_desc, void* stream);

/* ---- keyframe feature records of the reference's map files (csrc/orb_persist.hip) ---- */
/* SaveWorldToFile / LoadWroldFromFile (reference include/SaveLoadWorld.h:1254, 2463) store each
 * keyframe's features as one record per stream, little-endian as written on x86-64:
 *   keypoint stream (kfKeyPoints.bin, kfKeyPointsUn.bin; SaveLoadWorld.h:1406-1443, read back at
 *   2098-2160):   0xEB 0x90 | uint64 nKeys | nKeys x 28-byte cv::KeyPoint (= orb_keypoint_t)
 *   descriptor stream (kfDescriptors.bin; SaveLoadWorld.h:1446-1460, read back at 2166-2189):
 *                 0xEB 0x90 | int32 nDes | nDes x 32 bytes
 * Readers report a wrong header through *header_ok = 0 and go on, as the reference's loader
 * prints "header error ..., shouldn't" and keeps reading; a record longer than `len` is
 * ORB_ERANGE.  *consumed = bytes of the record (the next record starts there). */
size_t orb_keypoint_record_bytes(size_t n);
size_t orb_descriptor_record_bytes(int n);
int orb_write_keypoint_record(const orb_keypoint_t* kps, size_t n, uint8_t* out, size_t cap, size_t* written);
int orb_read_keypoint_record(const uint8_t* in, size_t len, orb_keypoint_t* kps, size_t cap, size_t* n,
                             size_t* consumed, int* header_ok);
int orb_write_descriptor_record(const uint8_t* desc, int n, uint8_t* out, size_t cap, size_t* written);
int orb_read_descriptor_record(const uint8_t* in, size_t len, uint8_t* desc, int cap, int* n, size_t* consumed,
                               int* header_ok);
/* B frames of orb_extract_batch_device output (per-frame capacity cap) packed on the device into
 * both streams, one record per frame in frame order (what SaveWorldToFile writes for B keyframes):
 * frame b's keypoint record at d_keys_stream + d_key_offsets[b], its descriptor record at
 * d_des_stream + d_des_offsets[b]; d_*_offsets[B] = the stream lengths (B + 1 int64 each).
 * keys_cap >= B * orb_keypoint_record_bytes(cap), des_cap >= B * orb_descriptor_record_bytes(cap);
 * buffers 2-byte aligned.  Asynchronous on `stream`. */
int orb_pack_keyframe_records_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                                     int cap, int B, uint8_t* d_keys_stream, size_t keys_cap, uint8_t* d_des_stream,
                                     size_t des_cap, int64_t* d_key_offsets, int64_t* d_des_offsets, void* stream);

/* ---- DBoW2 vocabulary (GPU: csrc/orb_voc.hip) -------------------------------------- */
/* The reference's ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (include/ORBVocabulary.h).  A handle holds the tree on `device`; host entry points are
 * serialised per handle, device entry points enqueue on the caller's stream.
 * Weighting: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY; scoring: 0 L1_NORM, 1 L2_NORM, 2 CHI_SQUARE,
 * 3 KL, 4 BHATTACHARYYA, 5 DOT_PRODUCT (BowVector.h:36-53). */
typedef struct orb_vocabulary orb_vocabulary_t; /* opaque handle */

/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424): header
 * "k L scoring weighting", then one line per node "parent isLeaf d0 .. d31 weight".
 * Blank lines are skipped; a malformed line or a parent that does not
 * precede its child is ORB_EINVAL (the reference reads such files unchecked). */
int orb_vocabulary_load_text(const char* path, int device, orb_vocabulary_t** out);
/* The same tree from arrays: node i + 1 (i < n_nodes) has parent[i] (<= i), is_leaf[i],
 * desc[32 i .. 32 i + 31] and weight[i], i.e. the lines of the text format in order. */
int orb_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                          const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                          orb_vocabulary_t** out);
int orb_vocabulary_destroy(orb_vocabulary_t* v);
/* info[7] = k, L, scoring, weighting, nodes (root included), words, tree height. */
int orb_vocabulary_info(const orb_vocabulary_t* v, int32_t* info);

/* transform(feature, word_id, weight, &nid, levelsup) (TemplatedVocabulary.h:1217-1259) for
 * n device descriptors (32 B rows, 16-B aligned): word id, weight and the node at level
 * L - levelsup (the root when that level is <= 0).  Asynchronous on `stream`. */
int orb_vocabulary_transform_features_device(const orb_vocabulary_t* v, int n, const uint8_t* d_desc, int levelsup,
                                             uint32_t* d_word, double* d_weight, uint32_t* d_node, void* stream);

/* transform(features, BowVector, FeatureVector, levelsup) (TemplatedVocabulary.h:1126-1194) for
 * B frames laid out as orb_extract_batch_device writes them (frame b: d_desc + b*cap*32,
 * d_counts[b] rows).  Per frame, capacity cap each: d_feat_* per-feature results (as above);
 * BowVector = d_bow_words / d_bow_values[d_bow_n[b]] in ascending word order; FeatureVector
 * = CSR d_fv_nodes[d_fv_n[b]], d_fv_offsets (cap + 1 per frame), d_fv_features.  cap <= 8192.
 * Asynchronous on `stream`. */
int orb_vocabulary_transform_batch_device(const orb_vocabulary_t* v, int B, const uint8_t* d_desc,
                                          const int32_t* d_counts, int cap, int levelsup, uint32_t* d_feat_word,
                                          double* d_feat_weight, uint32_t* d_feat_node, uint32_t* d_bow_words,
                                          double* d_bow_values, int32_t* d_bow_n, uint32_t* d_fv_nodes,
                                          int32_t* d_fv_offsets, int32_t* d_fv_features, int32_t* d_fv_n,
                                          void* stream);

/* The same for one frame of n host descriptors (synchronous); outputs sized n (offsets n + 1). */
int orb_vocabulary_transform(orb_vocabulary_t* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words,
                             double* bow_values, int* bow_n, uint32_t* fv_nodes, int32_t* fv_offsets,
                             int32_t* fv_features, int* fv_n);

/* ---- measurement ------------------------------------------------------------------- */
/* Per-stage HIP-event timing of the extraction kernels: when enabled, every
 * orb_extract_batch_device records an event pair around each stage on its launch stream.
 * orb_profile_read synchronises and returns cumulative milliseconds and launch counts per
 * stage (stage names via orb_profile_stage_name); the return value is the stage count.
 * Enabling (or re-enabling) resets the counters. */
int orb_profile_enable(orb_extractor_t* h, int enable);
/* The same for a subset of stages (bit k = stage k): every event pair is a stream boundary
 * (≈10 µs measured), so a timed run brackets only the stage it reports. */
int orb_profile_enable_stages(orb_extractor_t* h, unsigned stage_mask);
int orb_profile_read(orb_extractor_t* h, double* stage_ms, int64_t* stage_launches, int nstages);
const char* orb_profile_stage_name(int i);

/* Split orb_extract_batch_device into its two phases (scheduling only; results unchanged):
 * bit 0 = the image pyramid (ComputePyramid, ORBextractor.cc:781-822), bit 1 = detection,
 * selection, orientation and descriptors (ComputeKeyPoints + the descriptor loop,
 * ORBextractor.cc:522-707, 749-778), which read the pyramid that bit 0 left in the extractor's
 * workspace.  A caller running phase 1 then phase 2 for the same batch, on one stream or
 * event-ordered, gets exactly the mask-3 result; the gap between them lets other work (the
 * previous batch's matching) overlap the pyramid.  Default 3.  Applies to
 * orb_extract_batch_device only; every other extraction entry point runs both phases.
 * No reference counterpart. */
int orb_extract_set_phases(orb_extractor_t* h, unsigned phase_mask);

/* Test and diagnostic hooks (orb_debug_*): include/orb_debug.h. */

#ifdef __cplusplus
}
#endif
#endif /* ORB_ABI_H */
