/*
 * orb_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference ORB front end, used as the parity checker for the
 * HIP path (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only; the
 * product never links, loads or calls it).  See orb_oracle.cpp's header for what is
 * restated from where and how each un-vendored dependency is pinned.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H

#include <stdint.h>

#include "../include/orb_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_extractor oracle_extractor_t;

oracle_extractor_t* oracle_extractor_create(int nfeatures, float scale_factor, int nlevels, int score_type,
                                            int fast_th);
void oracle_extractor_destroy(oracle_extractor_t* h);
int oracle_get_level_info(const oracle_extractor_t* h, int* features_per_level, float* scale_factors,
                          float* inv_scale_factors, int* umax16);
/* ORBextractor::operator() on one image; returns status, *n_out keypoints. */
int oracle_extract(oracle_extractor_t* h, const uint8_t* img, int w, int hgt, int stride, orb_keypoint_t* kps,
                   int cap, uint8_t* desc, int* n_out);
/* After oracle_extract: padded (w+32)x(h+32) level `l` BEFORE the descriptor blur. */
int oracle_level_image(const oracle_extractor_t* h, int l, uint8_t* out, int* w, int* hgt);
/* After oracle_extract: the blurred ROI of level l (w x h), as the descriptors read it. */
int oracle_level_blurred(const oracle_extractor_t* h, int l, uint8_t* out);
/* After oracle_extract: per-cell FAST counts nTotal (row-major cells) of level l. */
int oracle_cell_counts(const oracle_extractor_t* h, int l, int* rows, int* cols, int* counts, int cap);

/* Primitives, exposed for unit tests. */
float oracle_fast_atan2(float y, float x);
float oracle_sinf(float x);
float oracle_cosf(float x);
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);
/* libstdc++ nth_element on float responses (greater): permutes idx[] of length n by keys. */
void oracle_nth_element_greater(const float* keys, int32_t* idx, int n, int nth);
/* OpenCV 2.4 getGaussianKernel(7, 2, CV_32F) * 256 -> int (the blur's fixed-point taps). */
void oracle_gaussian_taps(int* taps7);
/* ORBmatcher rotation-histogram bin of (a1 - a2) (ORBmatcher.cc:668-673). */
int oracle_rot_bin(float a1, float a2);
/* cv::resize(INTER_LINEAR) 8U restatement. */
int oracle_resize(const uint8_t* src, int sstep, int sw, int sh, uint8_t* dst, int dstep, int dw, int dh);
/* GaussianBlur(7x7, sigma 2) of the ROI of a (w+32) x (h+32) padded image (out: w x h). */
int oracle_blur_padded(const uint8_t* padded, int w, int hgt, uint8_t* out);
/* cv::FAST(img, kps, t, nonmax=true) on a region; out n x 3 (x, y, score); returns n. */
int oracle_fast(const uint8_t* img, int step, int cols, int rows, int threshold, int32_t* out, int cap);

int oracle_search_for_initialization(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1,
                                     const orb_keypoint_t* kps2, const uint8_t* desc2, int n2,
                                     orb_frame_bounds_t bounds, float nnratio, int check_ori, int window,
                                     float* prev_xy, int32_t* matches12, int* n_matches);

/* Frame::GetFeaturesInArea on a frame built from kps (reference Frame.cc:200-265). */
int oracle_features_in_area(const orb_keypoint_t* kps, int n, orb_frame_bounds_t bounds, float x, float y, float r,
                            int min_level, int max_level, int32_t* out, int cap);

/* SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:155-284).  FeatureVectors as CSR:
 * sorted node ids nodes[nn], offsets off[nn+1], feature indices feat[off[nn]].
 * kf_valid[i]: KF keypoint i has a non-bad MapPoint.  out_match[N_F]: KF feature index
 * whose MapPoint was assigned to F keypoint j, or -1. */
int oracle_search_by_bow_kf_f(const orb_keypoint_t* kf_kps, const uint8_t* kf_desc, int n_kf,
                              const uint8_t* kf_valid, const uint32_t* kf_nodes, const int32_t* kf_off,
                              const int32_t* kf_feat, int kf_nn, const orb_keypoint_t* f_kps, const uint8_t* f_desc,
                              int n_f, const uint32_t* f_nodes, const int32_t* f_off, const int32_t* f_feat, int f_nn,
                              float nnratio, int check_ori, int32_t* out_match, int* n_matches);

/* SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:715-850); out_match[n1] = idx2 or -1. */
int oracle_search_by_bow_kf_kf(const orb_keypoint_t* kps1, const uint8_t* desc1, int n1, const uint8_t* valid1,
                               const uint32_t* nodes1, const int32_t* off1, const int32_t* feat1, int nn1,
                               const orb_keypoint_t* kps2, const uint8_t* desc2, int n2, const uint8_t* valid2,
                               const uint32_t* nodes2, const int32_t* off2, const int32_t* feat2, int nn2,
                               float nnratio, int check_ori, int32_t* out_match, int* n_matches);

/* CPU baseline: extract B frames (frame k at imgs + k*pitch) with `threads` workers (one
 * extractor per worker, frames round-robin) and, if match != 0, SearchForInitialization on
 * consecutive pairs (t, t+1) with window 100.  Returns wall seconds (< 0 on error). */
double oracle_bench(int nfeatures, float scale_factor, int nlevels, int fast_th, const uint8_t* imgs, int B, int w,
                    int hgt, int stride, int64_t pitch, int threads, int match, int64_t* total_kps,
                    int64_t* total_matches);

/* ---- orb_oracle_match.cpp: the rest of the ORBmatcher family (same arguments as the
 * corresponding orb_* entry points of include/orb_abi.h, minus `device`) ---------------- */
int oracle_features_in_area_view(const orb_frame_view_t* view, int keyframe, float x, float y, float r, int min_level,
                                 int max_level, int32_t* out, int cap);
int oracle_frame_is_in_frustum(const orb_frame_view_t* F, orb_map_points_t mps, float viewing_cos_limit,
                               uint8_t* in_view, float* proj_x, float* proj_y, int32_t* level, float* view_cos);
int oracle_search_by_projection_local(const orb_frame_view_t* F, const uint8_t* f_taken, int n_mp,
                                      const uint8_t* usable, const float* proj_x, const float* proj_y,
                                      const int32_t* level, const float* view_cos, const uint8_t* mp_desc, float th,
                                      float nnratio, int32_t* f_match, int* n_matches);
int oracle_window_search(const orb_frame_view_t* F1, const uint8_t* usable1, const orb_frame_view_t* F2,
                         int window, int min_scale_level, int max_scale_level, float nnratio, int check_ori,
                         int32_t* match21, int* n_matches);
int oracle_search_by_projection_f2f(const orb_frame_view_t* F1, orb_map_points_t mp1, const uint8_t* usable1,
                                    const orb_frame_view_t* F2, const uint8_t* f2_taken, int window, float nnratio,
                                    int32_t* match2, int* n_matches);
int oracle_search_by_projection_motion(const orb_frame_view_t* Cur, const uint8_t* cur_taken,
                                       const orb_frame_view_t* Last, orb_map_points_t mp, const uint8_t* usable,
                                       float th, int check_ori, int32_t* cur_match, int* n_matches);
int oracle_search_by_projection_reloc(const orb_frame_view_t* Cur, const uint8_t* cur_taken,
                                      const orb_frame_view_t* KF, orb_map_points_t mp, const uint8_t* usable,
                                      float th, int orb_dist, int check_ori, int32_t* cur_match, int* n_matches);
int oracle_search_by_projection_sim3(const orb_frame_view_t* KF, const uint8_t* kf_taken, orb_map_points_t pts,
                                     const uint8_t* usable, int th, int32_t* kf_match, int* n_matches);
int oracle_fuse(const orb_frame_view_t* KF, orb_map_points_t pts, const uint8_t* usable, float th, int scw,
                int32_t* best_idx, int* n_fused);
int oracle_search_by_sim3(const orb_frame_view_t* KF1, orb_map_points_t mp1, const uint8_t* usable1,
                          const orb_frame_view_t* KF2, orb_map_points_t mp2, const uint8_t* usable2,
                          const float* sR12, const float* t12, const float* sR21, const float* t21, float th,
                          int32_t* match12, int* n_found);
int oracle_search_for_triangulation(const orb_frame_view_t* KF1, const uint8_t* has_mp1, orb_feature_vector_t fv1,
                                    const orb_frame_view_t* KF2, const uint8_t* has_mp2, orb_feature_vector_t fv2,
                                    const float* F12, float nnratio, int check_ori, int32_t* match12,
                                    int* n_matches);

/* ---- orb_oracle_frame.cpp: Frame::UndistortKeyPoints / ComputeImageBounds (Frame.cc:289-349),
 * cv::undistortPoints (OpenCV 2.4 cvUndistortPoints) restated.  K4 = (fx, fy, cx, cy),
 * dist4 = (k1, k2, p1, p2). ---------------------------------------------------------------- */
int oracle_undistort_points(const float* K4, const float* dist4, const float* xy, int n, float* out);
int oracle_undistort_keypoints(const orb_keypoint_t* kps, int n, const float* K4, const float* dist4,
                               orb_keypoint_t* out);
int oracle_compute_image_bounds(int cols, int rows, const float* K4, const float* dist4, orb_frame_bounds_t* b);

/* ---- orb_oracle_color.cpp: cvtColor(CV_RGB2GRAY / CV_BGR2GRAY) 8U (Tracking.cc:202-207) ---- */
int oracle_rgb_to_gray(const uint8_t* src, int w, int h, int stride, int cn, int rgb, uint8_t* dst);

/* ---- orb_oracle_mappoint.cpp: MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:185-250) */
int oracle_compute_distinctive_descriptors(int M, const int32_t* offsets, const uint8_t* desc, const uint8_t* usable,
                                           int32_t* best_row, uint8_t* out_desc);

/* ---- orb_oracle_voc.cpp: DBoW2 vocabulary (TemplatedVocabulary.h:1126-1259, 1338-1424) --- */
typedef struct oracle_vocabulary oracle_vocabulary_t;
oracle_vocabulary_t* oracle_vocabulary_load_text(const char* path);
oracle_vocabulary_t* oracle_vocabulary_create(int k, int L, int scoring, int weighting, int n_nodes,
                                              const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc,
                                              const double* weight);
void oracle_vocabulary_destroy(oracle_vocabulary_t* v);
/* info[6] = k, L, scoring, weighting, nodes (root included), words */
int oracle_vocabulary_info(const oracle_vocabulary_t* v, int32_t* info);
int oracle_vocabulary_transform_one(const oracle_vocabulary_t* v, const uint8_t* desc, int levelsup, uint32_t* word,
                                    double* weight, uint32_t* nid);
int oracle_vocabulary_transform(const oracle_vocabulary_t* v, const uint8_t* desc, int n, int levelsup,
                                uint32_t* bow_words, double* bow_values, int* bow_n, uint32_t* fv_nodes,
                                int32_t* fv_offsets, int32_t* fv_features, int* fv_n);

#ifdef __cplusplus
}
#endif
#endif
