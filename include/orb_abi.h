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
 *   stream: hipStream_t to enqueue on (NULL = the handle's own stream).  Asynchronous:
 *   returns after enqueueing; synchronise the stream before reading outputs. */
int orb_extract_batch_device(orb_extractor_t* h, int B, const uint8_t* d_imgs, int w, int hgt, int stride,
                             int64_t frame_pitch, orb_keypoint_t* d_kps, uint8_t* d_desc, int32_t* d_counts,
                             void* stream);

/* Host-buffer batch: copies B host frames in, runs, copies results out (synchronous).
 * kps_out / desc_out / n_out laid out as for the device variant. */
int orb_extract_batch(orb_extractor_t* h, int B, const uint8_t* imgs, int w, int hgt, int stride,
                      int64_t frame_pitch, orb_keypoint_t* kps_out, uint8_t* desc_out, int32_t* n_out);

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
 *   d_matches12: P x cap int32; d_nmatches: P int32.  Asynchronous on `stream`. */
int orb_search_for_initialization_batch_device(const orb_keypoint_t* d_kps, const uint8_t* d_desc,
                                               const int32_t* d_counts, int cap, int P, const int32_t* d_pair_f1,
                                               const int32_t* d_pair_f2, orb_frame_bounds_t bounds, float nnratio,
                                               int check_ori, int window, float* d_prev_xy, int32_t* d_matches12,
                                               int32_t* d_nmatches, void* stream);

/* ---- measurement ------------------------------------------------------------------- */
/* Per-stage HIP-event timing of the extraction kernels: when enabled, every
 * orb_extract_batch_device records an event pair around each stage on its launch stream.
 * orb_profile_read synchronises and returns cumulative milliseconds and launch counts per
 * stage (stage names via orb_profile_stage_name); the return value is the stage count.
 * Enabling (or re-enabling) resets the counters. */
int orb_profile_enable(orb_extractor_t* h, int enable);
int orb_profile_read(orb_extractor_t* h, double* stage_ms, int64_t* stage_launches, int nstages);
const char* orb_profile_stage_name(int i);

/* ---- test hooks (no device work unless stated) ------------------------------------- */
/* Host instantiation of the kernels' libstdc++ nth_element replay on packed u32 elements
 * (score in bits 24..31), for CPU unit tests against std::nth_element. */
int orb_debug_nth_element_u32(uint32_t* a, int n, int nth);
/* Padded pyramid level l of batch frame b after the last extraction (device sync). */
int orb_debug_level_image(orb_extractor_t* h, int b, int l, uint8_t* out, int* w, int* hgt);
/* Descriptor image (blurred ROI + un-blurred padding ring) of level l, frame b, padded
 * (w+32) x (h+32) layout; only the ring [-3, w+3) x [-3, h+3) is defined (device sync). */
int orb_debug_blur_image(orb_extractor_t* h, int b, int l, uint8_t* out);
/* Per-cell FAST keypoint counts of frame b, level l (device sync); returns #cells. */
int orb_debug_cell_counts(orb_extractor_t* h, int b, int l, int* counts, int cap);

#ifdef __cplusplus
}
#endif
#endif /* ORB_ABI_H */
