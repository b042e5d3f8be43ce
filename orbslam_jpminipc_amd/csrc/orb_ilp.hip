// orb_ilp.hip — k_fast and k_pyr_stream compiled with the machine scheduler's max-ILP strategy
// (`-mllvm -amdgpu-sched-strategy=max-ilp`: __graft_entry__.ILP_FLAGS, this unit only), launched
// by orb_hip.hip through the three functions below.
//
// Both kernels' occupancy is set by LDS (k_fast: five workgroups per CU) or by their own
// waves-per-EU target (k_pyr_stream: two workgroups per CU), so the default scheduler's
// occupancy-first schedule gains nothing from the registers it saves, and both kernels' time is
// their instruction issue: k_fast 442.5 -> 437.5 us per c3 step on one box, k_pyr_stream
// unchanged (289.4 / 289.9 us; both orders, two copies each: profiles/r06/r06_ilp3_summary.txt,
// HISTORY.md round 6).  The rest of
// the library keeps the default: k_orient_desc under max-ILP takes 112 VGPRs (occupancy 8 -> 4,
// 0.43 -> 0.58 ms) and spills when held to eight waves; k_select measured 10 % slower.
//
// The unit compiles orb_hip.hip again with ORB_TU_ILP: only the two kernels (and the device
// helpers and types they use) are defined, so their source stays the one in orb_hip.hip, which
// then leaves them out (ORB_ILP_SPLIT; 0 keeps both there and makes this unit empty).
#define ORB_TU_ILP 1
#include "orb_hip.hip"

#if ORB_ILP_SPLIT
__attribute__((visibility("hidden"))) void orb_ilp_init() {
    hipFuncSetAttribute((const void*)k_pyr_stream, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
}

__attribute__((visibility("hidden"))) void orb_ilp_pyr_stream(int B, size_t lds, hipStream_t st, const uint8_t* imgs,
                                                             int stride, long long fpitch, uint8_t* pyr,
                                                             const uint32_t* scol, const uint4* srows,
                                                             const StreamLevel* slv, const uint32_t* srounds,
                                                             const StreamGeom& sg, int* cellCount, int nCells) {
    hipLaunchKernelGGL(k_pyr_stream, dim3(B), dim3(PS_THREADS), lds, st, imgs, stride, fpitch, pyr, scol, srows, slv,
                       srounds, sg, cellCount, nCells);
}

__attribute__((visibility("hidden"))) void orb_ilp_fast(int nTiles, int B, hipStream_t st, const uint8_t* pyr,
                                                       const Geom& g, const FastTile* tiles, uint32_t* cand,
                                                       int* cellCount) {
    hipLaunchKernelGGL(k_fast, dim3(nTiles, B), dim3(256), 0, st, pyr, g, tiles, cand, cellCount);
}
#endif
