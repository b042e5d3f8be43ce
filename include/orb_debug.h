/* liborb_hip.so test and diagnostic hooks: NOT part of the reference's API surface.
 *
 * Exported by the product library so that the GPU parity tests can inspect intermediate
 * results (pyramid levels, the descriptor image, per-cell FAST counts), force a code path that
 * ordinary frames rarely reach (k_fast's plane-scan fallback, the per-level pyramid kernels) and
 * check the libstdc++ nth_element replays in isolation.  None of them changes a result.  The
 * per-phase timing probes of the kernels (orb_debug_{ps,km,kr,ks,kf}_timing) exist only in
 * experiment builds (-DPS_TIMING=1 etc.), never in the product library.
 */
#ifndef ORB_DEBUG_H
#define ORB_DEBUG_H
#include "orb_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- test hooks (no device work unless stated) ------------------------------------- */
/* Host instantiation of the kernels' libstdc++ nth_element replay on packed u32 elements
 * (score in bits 24..31), for CPU unit tests against std::nth_element. */
int orb_debug_nth_element_u32(uint32_t* a, int n, int nth);
/* The one-wave (ballot-partition) replay k_select uses, run on `device` (n <= 8192). */
int orb_debug_nth_element_wave_u32(uint32_t* a, int n, int nth, int device);
/* Padded pyramid level l of batch frame b after the last extraction (device sync). */
int orb_debug_level_image(orb_extractor_t* h, int b, int l, uint8_t* out, int* w, int* hgt);
/* Descriptor image (blurred ROI + un-blurred padding ring) of level l, frame b, padded
 * (w+32) x (h+32) layout; defined over [-3, w+3) x [-3, h+3) at least (wider where a dense
 * cell grid lets keypoints sit past the FAST border) (device sync). */
int orb_debug_blur_image(orb_extractor_t* h, int b, int l, uint8_t* out);
/* Per-cell FAST keypoint counts of frame b, level l (device sync); returns #cells. */
int orb_debug_cell_counts(orb_extractor_t* h, int b, int l, int* counts, int cap);
/* Pyramid kernels used by the next extractions (results are identical): 0 = automatic (the
 * one-pass streaming kernel k_pyr_stream for batches >= 256 grey frames, per-level launches
 * otherwise), 1 = per-level launches always, 2 = k_pyr_stream at every batch size of grey
 * frames whenever the current geometry has a stream plan. */
int orb_debug_set_pyramid_path(orb_extractor_t* h, int mode);
/* k_fast keeps each wave's corners in a list of up to 256 entries and falls back to scanning the
 * whole strength plane of its tile when a wave finds more; cap (0 .. 256) lowers that list's
 * capacity for the next extractions so the fallback runs on ordinary frames (results are
 * identical; test hook, tests/test_gpu_fast_fallback.py).  The default is 256. */
int orb_debug_set_fast_corner_list(orb_extractor_t* h, int cap);
/* The current geometry's k_pyr_stream plan: returns 1 (and level-0 rows per round, rounds,
 * LDS bytes) when there is one, 0 when the geometry only runs per-level launches. */
int orb_debug_pyramid_plan(const orb_extractor_t* h, int* rows_per_round, int* rounds, int* lds_bytes);

#ifdef __cplusplus
}
#endif
#endif /* ORB_DEBUG_H */
