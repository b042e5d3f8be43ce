// VALU issue rate per SIMD on gfx950 for the instruction kinds the extraction kernels use, at
// 1, 2, 4 and 8 waves per SIMD: does a wave64 integer / packed-16 / permute VALU op issue every
// 2 cycles per SIMD once several waves are resident (the SIMD-32 rate), or every 4?
// Each wave runs ITER x 16 instructions in 8 independent chains.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_rate scripts/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITER 4096

__global__ void __launch_bounds__(512) k_v_add_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_u32 %0, %0, %8\n"
"v_add_u32 %1, %1, %8\n"
"v_add_u32 %2, %2, %8\n"
"v_add_u32 %3, %3, %8\n"
"v_add_u32 %4, %4, %8\n"
"v_add_u32 %5, %5, %8\n"
"v_add_u32 %6, %6, %8\n"
"v_add_u32 %7, %7, %8\n"
"v_add_u32 %0, %0, %8\n"
"v_add_u32 %1, %1, %8\n"
"v_add_u32 %2, %2, %8\n"
"v_add_u32 %3, %3, %8\n"
"v_add_u32 %4, %4, %8\n"
"v_add_u32 %5, %5, %8\n"
"v_add_u32 %6, %6, %8\n"
"v_add_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_add_u32_e64(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_u32_e64 %0, %0, %8\n"
"v_add_u32_e64 %1, %1, %8\n"
"v_add_u32_e64 %2, %2, %8\n"
"v_add_u32_e64 %3, %3, %8\n"
"v_add_u32_e64 %4, %4, %8\n"
"v_add_u32_e64 %5, %5, %8\n"
"v_add_u32_e64 %6, %6, %8\n"
"v_add_u32_e64 %7, %7, %8\n"
"v_add_u32_e64 %0, %0, %8\n"
"v_add_u32_e64 %1, %1, %8\n"
"v_add_u32_e64 %2, %2, %8\n"
"v_add_u32_e64 %3, %3, %8\n"
"v_add_u32_e64 %4, %4, %8\n"
"v_add_u32_e64 %5, %5, %8\n"
"v_add_u32_e64 %6, %6, %8\n"
"v_add_u32_e64 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_sub_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_sub_u32 %0, %0, %8\n"
"v_sub_u32 %1, %1, %8\n"
"v_sub_u32 %2, %2, %8\n"
"v_sub_u32 %3, %3, %8\n"
"v_sub_u32 %4, %4, %8\n"
"v_sub_u32 %5, %5, %8\n"
"v_sub_u32 %6, %6, %8\n"
"v_sub_u32 %7, %7, %8\n"
"v_sub_u32 %0, %0, %8\n"
"v_sub_u32 %1, %1, %8\n"
"v_sub_u32 %2, %2, %8\n"
"v_sub_u32 %3, %3, %8\n"
"v_sub_u32 %4, %4, %8\n"
"v_sub_u32 %5, %5, %8\n"
"v_sub_u32 %6, %6, %8\n"
"v_sub_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_and_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_and_b32 %0, %0, %8\n"
"v_and_b32 %1, %1, %8\n"
"v_and_b32 %2, %2, %8\n"
"v_and_b32 %3, %3, %8\n"
"v_and_b32 %4, %4, %8\n"
"v_and_b32 %5, %5, %8\n"
"v_and_b32 %6, %6, %8\n"
"v_and_b32 %7, %7, %8\n"
"v_and_b32 %0, %0, %8\n"
"v_and_b32 %1, %1, %8\n"
"v_and_b32 %2, %2, %8\n"
"v_and_b32 %3, %3, %8\n"
"v_and_b32 %4, %4, %8\n"
"v_and_b32 %5, %5, %8\n"
"v_and_b32 %6, %6, %8\n"
"v_and_b32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_or_b32 %0, %0, %8\n"
"v_or_b32 %1, %1, %8\n"
"v_or_b32 %2, %2, %8\n"
"v_or_b32 %3, %3, %8\n"
"v_or_b32 %4, %4, %8\n"
"v_or_b32 %5, %5, %8\n"
"v_or_b32 %6, %6, %8\n"
"v_or_b32 %7, %7, %8\n"
"v_or_b32 %0, %0, %8\n"
"v_or_b32 %1, %1, %8\n"
"v_or_b32 %2, %2, %8\n"
"v_or_b32 %3, %3, %8\n"
"v_or_b32 %4, %4, %8\n"
"v_or_b32 %5, %5, %8\n"
"v_or_b32 %6, %6, %8\n"
"v_or_b32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_xor_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_xor_b32 %0, %0, %8\n"
"v_xor_b32 %1, %1, %8\n"
"v_xor_b32 %2, %2, %8\n"
"v_xor_b32 %3, %3, %8\n"
"v_xor_b32 %4, %4, %8\n"
"v_xor_b32 %5, %5, %8\n"
"v_xor_b32 %6, %6, %8\n"
"v_xor_b32 %7, %7, %8\n"
"v_xor_b32 %0, %0, %8\n"
"v_xor_b32 %1, %1, %8\n"
"v_xor_b32 %2, %2, %8\n"
"v_xor_b32 %3, %3, %8\n"
"v_xor_b32 %4, %4, %8\n"
"v_xor_b32 %5, %5, %8\n"
"v_xor_b32 %6, %6, %8\n"
"v_xor_b32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_lshrrev_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_lshrrev_b32 %0, %8, %0\n"
"v_lshrrev_b32 %1, %8, %1\n"
"v_lshrrev_b32 %2, %8, %2\n"
"v_lshrrev_b32 %3, %8, %3\n"
"v_lshrrev_b32 %4, %8, %4\n"
"v_lshrrev_b32 %5, %8, %5\n"
"v_lshrrev_b32 %6, %8, %6\n"
"v_lshrrev_b32 %7, %8, %7\n"
"v_lshrrev_b32 %0, %8, %0\n"
"v_lshrrev_b32 %1, %8, %1\n"
"v_lshrrev_b32 %2, %8, %2\n"
"v_lshrrev_b32 %3, %8, %3\n"
"v_lshrrev_b32 %4, %8, %4\n"
"v_lshrrev_b32 %5, %8, %5\n"
"v_lshrrev_b32 %6, %8, %6\n"
"v_lshrrev_b32 %7, %8, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_min_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_min_u32 %0, %0, %8\n"
"v_min_u32 %1, %1, %8\n"
"v_min_u32 %2, %2, %8\n"
"v_min_u32 %3, %3, %8\n"
"v_min_u32 %4, %4, %8\n"
"v_min_u32 %5, %5, %8\n"
"v_min_u32 %6, %6, %8\n"
"v_min_u32 %7, %7, %8\n"
"v_min_u32 %0, %0, %8\n"
"v_min_u32 %1, %1, %8\n"
"v_min_u32 %2, %2, %8\n"
"v_min_u32 %3, %3, %8\n"
"v_min_u32 %4, %4, %8\n"
"v_min_u32 %5, %5, %8\n"
"v_min_u32 %6, %6, %8\n"
"v_min_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_max_i32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_max_i32 %0, %0, %8\n"
"v_max_i32 %1, %1, %8\n"
"v_max_i32 %2, %2, %8\n"
"v_max_i32 %3, %3, %8\n"
"v_max_i32 %4, %4, %8\n"
"v_max_i32 %5, %5, %8\n"
"v_max_i32 %6, %6, %8\n"
"v_max_i32 %7, %7, %8\n"
"v_max_i32 %0, %0, %8\n"
"v_max_i32 %1, %1, %8\n"
"v_max_i32 %2, %2, %8\n"
"v_max_i32 %3, %3, %8\n"
"v_max_i32 %4, %4, %8\n"
"v_max_i32 %5, %5, %8\n"
"v_max_i32 %6, %6, %8\n"
"v_max_i32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_min_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_min_u16 %0, %0, %8\n"
"v_min_u16 %1, %1, %8\n"
"v_min_u16 %2, %2, %8\n"
"v_min_u16 %3, %3, %8\n"
"v_min_u16 %4, %4, %8\n"
"v_min_u16 %5, %5, %8\n"
"v_min_u16 %6, %6, %8\n"
"v_min_u16 %7, %7, %8\n"
"v_min_u16 %0, %0, %8\n"
"v_min_u16 %1, %1, %8\n"
"v_min_u16 %2, %2, %8\n"
"v_min_u16 %3, %3, %8\n"
"v_min_u16 %4, %4, %8\n"
"v_min_u16 %5, %5, %8\n"
"v_min_u16 %6, %6, %8\n"
"v_min_u16 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_mov_b32_dpp(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %5, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %6, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %7, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %5, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %6, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
"v_mov_b32_dpp %7, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_cndmask_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n"
"v_cndmask_b32 %1, %1, %8, vcc\n"
"v_cndmask_b32 %2, %2, %8, vcc\n"
"v_cndmask_b32 %3, %3, %8, vcc\n"
"v_cndmask_b32 %4, %4, %8, vcc\n"
"v_cndmask_b32 %5, %5, %8, vcc\n"
"v_cndmask_b32 %6, %6, %8, vcc\n"
"v_cndmask_b32 %7, %7, %8, vcc\n"
"v_cndmask_b32 %0, %0, %8, vcc\n"
"v_cndmask_b32 %1, %1, %8, vcc\n"
"v_cndmask_b32 %2, %2, %8, vcc\n"
"v_cndmask_b32 %3, %3, %8, vcc\n"
"v_cndmask_b32 %4, %4, %8, vcc\n"
"v_cndmask_b32 %5, %5, %8, vcc\n"
"v_cndmask_b32 %6, %6, %8, vcc\n"
"v_cndmask_b32 %7, %7, %8, vcc\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_add_f32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_f32 %0, %0, %8\n"
"v_add_f32 %1, %1, %8\n"
"v_add_f32 %2, %2, %8\n"
"v_add_f32 %3, %3, %8\n"
"v_add_f32 %4, %4, %8\n"
"v_add_f32 %5, %5, %8\n"
"v_add_f32 %6, %6, %8\n"
"v_add_f32 %7, %7, %8\n"
"v_add_f32 %0, %0, %8\n"
"v_add_f32 %1, %1, %8\n"
"v_add_f32 %2, %2, %8\n"
"v_add_f32 %3, %3, %8\n"
"v_add_f32 %4, %4, %8\n"
"v_add_f32 %5, %5, %8\n"
"v_add_f32 %6, %6, %8\n"
"v_add_f32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_mul_f32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mul_f32 %0, %0, %8\n"
"v_mul_f32 %1, %1, %8\n"
"v_mul_f32 %2, %2, %8\n"
"v_mul_f32 %3, %3, %8\n"
"v_mul_f32 %4, %4, %8\n"
"v_mul_f32 %5, %5, %8\n"
"v_mul_f32 %6, %6, %8\n"
"v_mul_f32 %7, %7, %8\n"
"v_mul_f32 %0, %0, %8\n"
"v_mul_f32 %1, %1, %8\n"
"v_mul_f32 %2, %2, %8\n"
"v_mul_f32 %3, %3, %8\n"
"v_mul_f32 %4, %4, %8\n"
"v_mul_f32 %5, %5, %8\n"
"v_mul_f32 %6, %6, %8\n"
"v_mul_f32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_fmac_f32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_fmac_f32 %0, %8, %9\n"
"v_fmac_f32 %1, %8, %9\n"
"v_fmac_f32 %2, %8, %9\n"
"v_fmac_f32 %3, %8, %9\n"
"v_fmac_f32 %4, %8, %9\n"
"v_fmac_f32 %5, %8, %9\n"
"v_fmac_f32 %6, %8, %9\n"
"v_fmac_f32 %7, %8, %9\n"
"v_fmac_f32 %0, %8, %9\n"
"v_fmac_f32 %1, %8, %9\n"
"v_fmac_f32 %2, %8, %9\n"
"v_fmac_f32 %3, %8, %9\n"
"v_fmac_f32 %4, %8, %9\n"
"v_fmac_f32 %5, %8, %9\n"
"v_fmac_f32 %6, %8, %9\n"
"v_fmac_f32 %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_fma_f32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_fma_f32 %0, %0, %8, %9\n"
"v_fma_f32 %1, %1, %8, %9\n"
"v_fma_f32 %2, %2, %8, %9\n"
"v_fma_f32 %3, %3, %8, %9\n"
"v_fma_f32 %4, %4, %8, %9\n"
"v_fma_f32 %5, %5, %8, %9\n"
"v_fma_f32 %6, %6, %8, %9\n"
"v_fma_f32 %7, %7, %8, %9\n"
"v_fma_f32 %0, %0, %8, %9\n"
"v_fma_f32 %1, %1, %8, %9\n"
"v_fma_f32 %2, %2, %8, %9\n"
"v_fma_f32 %3, %3, %8, %9\n"
"v_fma_f32 %4, %4, %8, %9\n"
"v_fma_f32 %5, %5, %8, %9\n"
"v_fma_f32 %6, %6, %8, %9\n"
"v_fma_f32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_pk_fma_f32(uint32_t* out, uint32_t seed) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 r[8];
    for (int q = 0; q < 8; ++q) r[q] = f2{(float)(threadIdx.x ^ seed) + q, 1.0f};
    const f2 k = f2{1.0f, (float)seed};
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_fma_f32 %0, %0, %10, %10\n"
"v_pk_fma_f32 %1, %1, %10, %10\n"
"v_pk_fma_f32 %2, %2, %10, %10\n"
"v_pk_fma_f32 %3, %3, %10, %10\n"
"v_pk_fma_f32 %4, %4, %10, %10\n"
"v_pk_fma_f32 %5, %5, %10, %10\n"
"v_pk_fma_f32 %6, %6, %10, %10\n"
"v_pk_fma_f32 %7, %7, %10, %10\n"
"v_pk_fma_f32 %0, %0, %10, %10\n"
"v_pk_fma_f32 %1, %1, %10, %10\n"
"v_pk_fma_f32 %2, %2, %10, %10\n"
"v_pk_fma_f32 %3, %3, %10, %10\n"
"v_pk_fma_f32 %4, %4, %10, %10\n"
"v_pk_fma_f32 %5, %5, %10, %10\n"
"v_pk_fma_f32 %6, %6, %10, %10\n"
"v_pk_fma_f32 %7, %7, %10, %10\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(seed), "v"(seed), "v"(k));
    }
    float a = 0;
    for (int q = 0; q < 8; ++q) a += r[q].x + r[q].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(a);
}
__global__ void __launch_bounds__(512) k_v_mul_u32_u24(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mul_u32_u24 %0, %0, %8\n"
"v_mul_u32_u24 %1, %1, %8\n"
"v_mul_u32_u24 %2, %2, %8\n"
"v_mul_u32_u24 %3, %3, %8\n"
"v_mul_u32_u24 %4, %4, %8\n"
"v_mul_u32_u24 %5, %5, %8\n"
"v_mul_u32_u24 %6, %6, %8\n"
"v_mul_u32_u24 %7, %7, %8\n"
"v_mul_u32_u24 %0, %0, %8\n"
"v_mul_u32_u24 %1, %1, %8\n"
"v_mul_u32_u24 %2, %2, %8\n"
"v_mul_u32_u24 %3, %3, %8\n"
"v_mul_u32_u24 %4, %4, %8\n"
"v_mul_u32_u24 %5, %5, %8\n"
"v_mul_u32_u24 %6, %6, %8\n"
"v_mul_u32_u24 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_mul_hi_u32_u24(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %8\n"
"v_mul_hi_u32_u24 %1, %1, %8\n"
"v_mul_hi_u32_u24 %2, %2, %8\n"
"v_mul_hi_u32_u24 %3, %3, %8\n"
"v_mul_hi_u32_u24 %4, %4, %8\n"
"v_mul_hi_u32_u24 %5, %5, %8\n"
"v_mul_hi_u32_u24 %6, %6, %8\n"
"v_mul_hi_u32_u24 %7, %7, %8\n"
"v_mul_hi_u32_u24 %0, %0, %8\n"
"v_mul_hi_u32_u24 %1, %1, %8\n"
"v_mul_hi_u32_u24 %2, %2, %8\n"
"v_mul_hi_u32_u24 %3, %3, %8\n"
"v_mul_hi_u32_u24 %4, %4, %8\n"
"v_mul_hi_u32_u24 %5, %5, %8\n"
"v_mul_hi_u32_u24 %6, %6, %8\n"
"v_mul_hi_u32_u24 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_mad_u32_u24(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mad_u32_u24 %0, %0, %8, %9\n"
"v_mad_u32_u24 %1, %1, %8, %9\n"
"v_mad_u32_u24 %2, %2, %8, %9\n"
"v_mad_u32_u24 %3, %3, %8, %9\n"
"v_mad_u32_u24 %4, %4, %8, %9\n"
"v_mad_u32_u24 %5, %5, %8, %9\n"
"v_mad_u32_u24 %6, %6, %8, %9\n"
"v_mad_u32_u24 %7, %7, %8, %9\n"
"v_mad_u32_u24 %0, %0, %8, %9\n"
"v_mad_u32_u24 %1, %1, %8, %9\n"
"v_mad_u32_u24 %2, %2, %8, %9\n"
"v_mad_u32_u24 %3, %3, %8, %9\n"
"v_mad_u32_u24 %4, %4, %8, %9\n"
"v_mad_u32_u24 %5, %5, %8, %9\n"
"v_mad_u32_u24 %6, %6, %8, %9\n"
"v_mad_u32_u24 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_mul_lo_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mul_lo_u32 %0, %0, %8\n"
"v_mul_lo_u32 %1, %1, %8\n"
"v_mul_lo_u32 %2, %2, %8\n"
"v_mul_lo_u32 %3, %3, %8\n"
"v_mul_lo_u32 %4, %4, %8\n"
"v_mul_lo_u32 %5, %5, %8\n"
"v_mul_lo_u32 %6, %6, %8\n"
"v_mul_lo_u32 %7, %7, %8\n"
"v_mul_lo_u32 %0, %0, %8\n"
"v_mul_lo_u32 %1, %1, %8\n"
"v_mul_lo_u32 %2, %2, %8\n"
"v_mul_lo_u32 %3, %3, %8\n"
"v_mul_lo_u32 %4, %4, %8\n"
"v_mul_lo_u32 %5, %5, %8\n"
"v_mul_lo_u32 %6, %6, %8\n"
"v_mul_lo_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_bfe_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_bfe_u32 %0, %0, 3, 8\n"
"v_bfe_u32 %1, %1, 3, 8\n"
"v_bfe_u32 %2, %2, 3, 8\n"
"v_bfe_u32 %3, %3, 3, 8\n"
"v_bfe_u32 %4, %4, 3, 8\n"
"v_bfe_u32 %5, %5, 3, 8\n"
"v_bfe_u32 %6, %6, 3, 8\n"
"v_bfe_u32 %7, %7, 3, 8\n"
"v_bfe_u32 %0, %0, 3, 8\n"
"v_bfe_u32 %1, %1, 3, 8\n"
"v_bfe_u32 %2, %2, 3, 8\n"
"v_bfe_u32 %3, %3, 3, 8\n"
"v_bfe_u32 %4, %4, 3, 8\n"
"v_bfe_u32 %5, %5, 3, 8\n"
"v_bfe_u32 %6, %6, 3, 8\n"
"v_bfe_u32 %7, %7, 3, 8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_bfi_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_bfi_b32 %0, %0, %8, %9\n"
"v_bfi_b32 %1, %1, %8, %9\n"
"v_bfi_b32 %2, %2, %8, %9\n"
"v_bfi_b32 %3, %3, %8, %9\n"
"v_bfi_b32 %4, %4, %8, %9\n"
"v_bfi_b32 %5, %5, %8, %9\n"
"v_bfi_b32 %6, %6, %8, %9\n"
"v_bfi_b32 %7, %7, %8, %9\n"
"v_bfi_b32 %0, %0, %8, %9\n"
"v_bfi_b32 %1, %1, %8, %9\n"
"v_bfi_b32 %2, %2, %8, %9\n"
"v_bfi_b32 %3, %3, %8, %9\n"
"v_bfi_b32 %4, %4, %8, %9\n"
"v_bfi_b32 %5, %5, %8, %9\n"
"v_bfi_b32 %6, %6, %8, %9\n"
"v_bfi_b32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_alignbyte_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_alignbyte_b32 %0, %0, %8, 1\n"
"v_alignbyte_b32 %1, %1, %8, 1\n"
"v_alignbyte_b32 %2, %2, %8, 1\n"
"v_alignbyte_b32 %3, %3, %8, 1\n"
"v_alignbyte_b32 %4, %4, %8, 1\n"
"v_alignbyte_b32 %5, %5, %8, 1\n"
"v_alignbyte_b32 %6, %6, %8, 1\n"
"v_alignbyte_b32 %7, %7, %8, 1\n"
"v_alignbyte_b32 %0, %0, %8, 1\n"
"v_alignbyte_b32 %1, %1, %8, 1\n"
"v_alignbyte_b32 %2, %2, %8, 1\n"
"v_alignbyte_b32 %3, %3, %8, 1\n"
"v_alignbyte_b32 %4, %4, %8, 1\n"
"v_alignbyte_b32 %5, %5, %8, 1\n"
"v_alignbyte_b32 %6, %6, %8, 1\n"
"v_alignbyte_b32 %7, %7, %8, 1\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_perm_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_perm_b32 %0, %0, %8, %9\n"
"v_perm_b32 %1, %1, %8, %9\n"
"v_perm_b32 %2, %2, %8, %9\n"
"v_perm_b32 %3, %3, %8, %9\n"
"v_perm_b32 %4, %4, %8, %9\n"
"v_perm_b32 %5, %5, %8, %9\n"
"v_perm_b32 %6, %6, %8, %9\n"
"v_perm_b32 %7, %7, %8, %9\n"
"v_perm_b32 %0, %0, %8, %9\n"
"v_perm_b32 %1, %1, %8, %9\n"
"v_perm_b32 %2, %2, %8, %9\n"
"v_perm_b32 %3, %3, %8, %9\n"
"v_perm_b32 %4, %4, %8, %9\n"
"v_perm_b32 %5, %5, %8, %9\n"
"v_perm_b32 %6, %6, %8, %9\n"
"v_perm_b32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_add3_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add3_u32 %0, %0, %8, %9\n"
"v_add3_u32 %1, %1, %8, %9\n"
"v_add3_u32 %2, %2, %8, %9\n"
"v_add3_u32 %3, %3, %8, %9\n"
"v_add3_u32 %4, %4, %8, %9\n"
"v_add3_u32 %5, %5, %8, %9\n"
"v_add3_u32 %6, %6, %8, %9\n"
"v_add3_u32 %7, %7, %8, %9\n"
"v_add3_u32 %0, %0, %8, %9\n"
"v_add3_u32 %1, %1, %8, %9\n"
"v_add3_u32 %2, %2, %8, %9\n"
"v_add3_u32 %3, %3, %8, %9\n"
"v_add3_u32 %4, %4, %8, %9\n"
"v_add3_u32 %5, %5, %8, %9\n"
"v_add3_u32 %6, %6, %8, %9\n"
"v_add3_u32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_lshl_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %8\n"
"v_lshl_or_b32 %1, %1, 3, %8\n"
"v_lshl_or_b32 %2, %2, 3, %8\n"
"v_lshl_or_b32 %3, %3, 3, %8\n"
"v_lshl_or_b32 %4, %4, 3, %8\n"
"v_lshl_or_b32 %5, %5, 3, %8\n"
"v_lshl_or_b32 %6, %6, 3, %8\n"
"v_lshl_or_b32 %7, %7, 3, %8\n"
"v_lshl_or_b32 %0, %0, 3, %8\n"
"v_lshl_or_b32 %1, %1, 3, %8\n"
"v_lshl_or_b32 %2, %2, 3, %8\n"
"v_lshl_or_b32 %3, %3, 3, %8\n"
"v_lshl_or_b32 %4, %4, 3, %8\n"
"v_lshl_or_b32 %5, %5, 3, %8\n"
"v_lshl_or_b32 %6, %6, 3, %8\n"
"v_lshl_or_b32 %7, %7, 3, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_and_or_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_and_or_b32 %0, %0, %8, %9\n"
"v_and_or_b32 %1, %1, %8, %9\n"
"v_and_or_b32 %2, %2, %8, %9\n"
"v_and_or_b32 %3, %3, %8, %9\n"
"v_and_or_b32 %4, %4, %8, %9\n"
"v_and_or_b32 %5, %5, %8, %9\n"
"v_and_or_b32 %6, %6, %8, %9\n"
"v_and_or_b32 %7, %7, %8, %9\n"
"v_and_or_b32 %0, %0, %8, %9\n"
"v_and_or_b32 %1, %1, %8, %9\n"
"v_and_or_b32 %2, %2, %8, %9\n"
"v_and_or_b32 %3, %3, %8, %9\n"
"v_and_or_b32 %4, %4, %8, %9\n"
"v_and_or_b32 %5, %5, %8, %9\n"
"v_and_or_b32 %6, %6, %8, %9\n"
"v_and_or_b32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_min3_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_min3_u32 %0, %0, %8, %9\n"
"v_min3_u32 %1, %1, %8, %9\n"
"v_min3_u32 %2, %2, %8, %9\n"
"v_min3_u32 %3, %3, %8, %9\n"
"v_min3_u32 %4, %4, %8, %9\n"
"v_min3_u32 %5, %5, %8, %9\n"
"v_min3_u32 %6, %6, %8, %9\n"
"v_min3_u32 %7, %7, %8, %9\n"
"v_min3_u32 %0, %0, %8, %9\n"
"v_min3_u32 %1, %1, %8, %9\n"
"v_min3_u32 %2, %2, %8, %9\n"
"v_min3_u32 %3, %3, %8, %9\n"
"v_min3_u32 %4, %4, %8, %9\n"
"v_min3_u32 %5, %5, %8, %9\n"
"v_min3_u32 %6, %6, %8, %9\n"
"v_min3_u32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_med3_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_med3_u32 %0, %0, %8, %9\n"
"v_med3_u32 %1, %1, %8, %9\n"
"v_med3_u32 %2, %2, %8, %9\n"
"v_med3_u32 %3, %3, %8, %9\n"
"v_med3_u32 %4, %4, %8, %9\n"
"v_med3_u32 %5, %5, %8, %9\n"
"v_med3_u32 %6, %6, %8, %9\n"
"v_med3_u32 %7, %7, %8, %9\n"
"v_med3_u32 %0, %0, %8, %9\n"
"v_med3_u32 %1, %1, %8, %9\n"
"v_med3_u32 %2, %2, %8, %9\n"
"v_med3_u32 %3, %3, %8, %9\n"
"v_med3_u32 %4, %4, %8, %9\n"
"v_med3_u32 %5, %5, %8, %9\n"
"v_med3_u32 %6, %6, %8, %9\n"
"v_med3_u32 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_sad_u8(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_sad_u8 %0, %0, %8, %9\n"
"v_sad_u8 %1, %1, %8, %9\n"
"v_sad_u8 %2, %2, %8, %9\n"
"v_sad_u8 %3, %3, %8, %9\n"
"v_sad_u8 %4, %4, %8, %9\n"
"v_sad_u8 %5, %5, %8, %9\n"
"v_sad_u8 %6, %6, %8, %9\n"
"v_sad_u8 %7, %7, %8, %9\n"
"v_sad_u8 %0, %0, %8, %9\n"
"v_sad_u8 %1, %1, %8, %9\n"
"v_sad_u8 %2, %2, %8, %9\n"
"v_sad_u8 %3, %3, %8, %9\n"
"v_sad_u8 %4, %4, %8, %9\n"
"v_sad_u8 %5, %5, %8, %9\n"
"v_sad_u8 %6, %6, %8, %9\n"
"v_sad_u8 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_pk_min_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_min_u16 %0, %0, %8\n"
"v_pk_min_u16 %1, %1, %8\n"
"v_pk_min_u16 %2, %2, %8\n"
"v_pk_min_u16 %3, %3, %8\n"
"v_pk_min_u16 %4, %4, %8\n"
"v_pk_min_u16 %5, %5, %8\n"
"v_pk_min_u16 %6, %6, %8\n"
"v_pk_min_u16 %7, %7, %8\n"
"v_pk_min_u16 %0, %0, %8\n"
"v_pk_min_u16 %1, %1, %8\n"
"v_pk_min_u16 %2, %2, %8\n"
"v_pk_min_u16 %3, %3, %8\n"
"v_pk_min_u16 %4, %4, %8\n"
"v_pk_min_u16 %5, %5, %8\n"
"v_pk_min_u16 %6, %6, %8\n"
"v_pk_min_u16 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_pk_add_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_add_u16 %0, %0, %8\n"
"v_pk_add_u16 %1, %1, %8\n"
"v_pk_add_u16 %2, %2, %8\n"
"v_pk_add_u16 %3, %3, %8\n"
"v_pk_add_u16 %4, %4, %8\n"
"v_pk_add_u16 %5, %5, %8\n"
"v_pk_add_u16 %6, %6, %8\n"
"v_pk_add_u16 %7, %7, %8\n"
"v_pk_add_u16 %0, %0, %8\n"
"v_pk_add_u16 %1, %1, %8\n"
"v_pk_add_u16 %2, %2, %8\n"
"v_pk_add_u16 %3, %3, %8\n"
"v_pk_add_u16 %4, %4, %8\n"
"v_pk_add_u16 %5, %5, %8\n"
"v_pk_add_u16 %6, %6, %8\n"
"v_pk_add_u16 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_pk_add_f16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_add_f16 %0, %0, %8\n"
"v_pk_add_f16 %1, %1, %8\n"
"v_pk_add_f16 %2, %2, %8\n"
"v_pk_add_f16 %3, %3, %8\n"
"v_pk_add_f16 %4, %4, %8\n"
"v_pk_add_f16 %5, %5, %8\n"
"v_pk_add_f16 %6, %6, %8\n"
"v_pk_add_f16 %7, %7, %8\n"
"v_pk_add_f16 %0, %0, %8\n"
"v_pk_add_f16 %1, %1, %8\n"
"v_pk_add_f16 %2, %2, %8\n"
"v_pk_add_f16 %3, %3, %8\n"
"v_pk_add_f16 %4, %4, %8\n"
"v_pk_add_f16 %5, %5, %8\n"
"v_pk_add_f16 %6, %6, %8\n"
"v_pk_add_f16 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_pk_minimum3_f16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_minimum3_f16 %0, %0, %8, %9\n"
"v_pk_minimum3_f16 %1, %1, %8, %9\n"
"v_pk_minimum3_f16 %2, %2, %8, %9\n"
"v_pk_minimum3_f16 %3, %3, %8, %9\n"
"v_pk_minimum3_f16 %4, %4, %8, %9\n"
"v_pk_minimum3_f16 %5, %5, %8, %9\n"
"v_pk_minimum3_f16 %6, %6, %8, %9\n"
"v_pk_minimum3_f16 %7, %7, %8, %9\n"
"v_pk_minimum3_f16 %0, %0, %8, %9\n"
"v_pk_minimum3_f16 %1, %1, %8, %9\n"
"v_pk_minimum3_f16 %2, %2, %8, %9\n"
"v_pk_minimum3_f16 %3, %3, %8, %9\n"
"v_pk_minimum3_f16 %4, %4, %8, %9\n"
"v_pk_minimum3_f16 %5, %5, %8, %9\n"
"v_pk_minimum3_f16 %6, %6, %8, %9\n"
"v_pk_minimum3_f16 %7, %7, %8, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_dot4_u32_u8(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_dot4_u32_u8 %0, %0, %8, %0\n"
"v_dot4_u32_u8 %1, %1, %8, %1\n"
"v_dot4_u32_u8 %2, %2, %8, %2\n"
"v_dot4_u32_u8 %3, %3, %8, %3\n"
"v_dot4_u32_u8 %4, %4, %8, %4\n"
"v_dot4_u32_u8 %5, %5, %8, %5\n"
"v_dot4_u32_u8 %6, %6, %8, %6\n"
"v_dot4_u32_u8 %7, %7, %8, %7\n"
"v_dot4_u32_u8 %0, %0, %8, %0\n"
"v_dot4_u32_u8 %1, %1, %8, %1\n"
"v_dot4_u32_u8 %2, %2, %8, %2\n"
"v_dot4_u32_u8 %3, %3, %8, %3\n"
"v_dot4_u32_u8 %4, %4, %8, %4\n"
"v_dot4_u32_u8 %5, %5, %8, %5\n"
"v_dot4_u32_u8 %6, %6, %8, %6\n"
"v_dot4_u32_u8 %7, %7, %8, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_dot2_u32_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_dot2_u32_u16 %0, %0, %8, %0\n"
"v_dot2_u32_u16 %1, %1, %8, %1\n"
"v_dot2_u32_u16 %2, %2, %8, %2\n"
"v_dot2_u32_u16 %3, %3, %8, %3\n"
"v_dot2_u32_u16 %4, %4, %8, %4\n"
"v_dot2_u32_u16 %5, %5, %8, %5\n"
"v_dot2_u32_u16 %6, %6, %8, %6\n"
"v_dot2_u32_u16 %7, %7, %8, %7\n"
"v_dot2_u32_u16 %0, %0, %8, %0\n"
"v_dot2_u32_u16 %1, %1, %8, %1\n"
"v_dot2_u32_u16 %2, %2, %8, %2\n"
"v_dot2_u32_u16 %3, %3, %8, %3\n"
"v_dot2_u32_u16 %4, %4, %8, %4\n"
"v_dot2_u32_u16 %5, %5, %8, %5\n"
"v_dot2_u32_u16 %6, %6, %8, %6\n"
"v_dot2_u32_u16 %7, %7, %8, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_v_cvt_f32_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_cvt_f32_u32 %0, %0\n"
"v_cvt_f32_u32 %1, %1\n"
"v_cvt_f32_u32 %2, %2\n"
"v_cvt_f32_u32 %3, %3\n"
"v_cvt_f32_u32 %4, %4\n"
"v_cvt_f32_u32 %5, %5\n"
"v_cvt_f32_u32 %6, %6\n"
"v_cvt_f32_u32 %7, %7\n"
"v_cvt_f32_u32 %0, %0\n"
"v_cvt_f32_u32 %1, %1\n"
"v_cvt_f32_u32 %2, %2\n"
"v_cvt_f32_u32 %3, %3\n"
"v_cvt_f32_u32 %4, %4\n"
"v_cvt_f32_u32 %5, %5\n"
"v_cvt_f32_u32 %6, %6\n"
"v_cvt_f32_u32 %7, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2), "v"((double)k) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_mix_perm_add(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_perm_b32 %0, %0, %8, %9\n"
"v_add_u32 %1, %1, %8\n"
"v_perm_b32 %2, %2, %8, %9\n"
"v_add_u32 %3, %3, %8\n"
"v_perm_b32 %4, %4, %8, %9\n"
"v_add_u32 %5, %5, %8\n"
"v_perm_b32 %6, %6, %8, %9\n"
"v_add_u32 %7, %7, %8\n"
"v_perm_b32 %0, %0, %8, %9\n"
"v_add_u32 %1, %1, %8\n"
"v_perm_b32 %2, %2, %8, %9\n"
"v_add_u32 %3, %3, %8\n"
"v_perm_b32 %4, %4, %8, %9\n"
"v_add_u32 %5, %5, %8\n"
"v_perm_b32 %6, %6, %8, %9\n"
"v_add_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_mix_pkmin_and(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_pk_min_u16 %0, %0, %8\n"
"v_and_b32 %1, %1, %8\n"
"v_pk_min_u16 %2, %2, %8\n"
"v_and_b32 %3, %3, %8\n"
"v_pk_min_u16 %4, %4, %8\n"
"v_and_b32 %5, %5, %8\n"
"v_pk_min_u16 %6, %6, %8\n"
"v_and_b32 %7, %7, %8\n"
"v_pk_min_u16 %0, %0, %8\n"
"v_and_b32 %1, %1, %8\n"
"v_pk_min_u16 %2, %2, %8\n"
"v_and_b32 %3, %3, %8\n"
"v_pk_min_u16 %4, %4, %8\n"
"v_and_b32 %5, %5, %8\n"
"v_pk_min_u16 %6, %6, %8\n"
"v_and_b32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}
__global__ void __launch_bounds__(512) k_mix_dot4_add(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_dot4_u32_u8 %0, %0, %8, %0\n"
"v_add_u32 %1, %1, %8\n"
"v_dot4_u32_u8 %2, %2, %8, %2\n"
"v_add_u32 %3, %3, %8\n"
"v_dot4_u32_u8 %4, %4, %8, %4\n"
"v_add_u32 %5, %5, %8\n"
"v_dot4_u32_u8 %6, %6, %8, %6\n"
"v_add_u32 %7, %7, %8\n"
"v_dot4_u32_u8 %0, %0, %8, %0\n"
"v_add_u32 %1, %1, %8\n"
"v_dot4_u32_u8 %2, %2, %8, %2\n"
"v_add_u32 %3, %3, %8\n"
"v_dot4_u32_u8 %4, %4, %8, %4\n"
"v_add_u32 %5, %5, %8\n"
"v_dot4_u32_u8 %6, %6, %8, %6\n"
"v_add_u32 %7, %7, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                     : "v"(k), "v"(k2));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
}

__global__ void __launch_bounds__(512) k_v_cndmask_b32_e64(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %9, %8\n"
"v_cndmask_b32_e64 %1, %1, %9, %8\n"
"v_cndmask_b32_e64 %2, %2, %9, %8\n"
"v_cndmask_b32_e64 %3, %3, %9, %8\n"
"v_cndmask_b32_e64 %4, %4, %9, %8\n"
"v_cndmask_b32_e64 %5, %5, %9, %8\n"
"v_cndmask_b32_e64 %6, %6, %9, %8\n"
"v_cndmask_b32_e64 %7, %7, %9, %8\n"
"v_cndmask_b32_e64 %0, %0, %9, %8\n"
"v_cndmask_b32_e64 %1, %1, %9, %8\n"
"v_cndmask_b32_e64 %2, %2, %9, %8\n"
"v_cndmask_b32_e64 %3, %3, %9, %8\n"
"v_cndmask_b32_e64 %4, %4, %9, %8\n"
"v_cndmask_b32_e64 %5, %5, %9, %8\n"
"v_cndmask_b32_e64 %6, %6, %9, %8\n"
"v_cndmask_b32_e64 %7, %7, %9, %8\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_cndmask_b32_vcc_set(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
        asm volatile("v_cndmask_b32 %0, %0, %9, vcc\n"
"v_cndmask_b32 %1, %1, %9, vcc\n"
"v_cndmask_b32 %2, %2, %9, vcc\n"
"v_cndmask_b32 %3, %3, %9, vcc\n"
"v_cndmask_b32 %4, %4, %9, vcc\n"
"v_cndmask_b32 %5, %5, %9, vcc\n"
"v_cndmask_b32 %6, %6, %9, vcc\n"
"v_cndmask_b32 %7, %7, %9, vcc\n"
"v_cndmask_b32 %0, %0, %9, vcc\n"
"v_cndmask_b32 %1, %1, %9, vcc\n"
"v_cndmask_b32 %2, %2, %9, vcc\n"
"v_cndmask_b32 %3, %3, %9, vcc\n"
"v_cndmask_b32 %4, %4, %9, vcc\n"
"v_cndmask_b32 %5, %5, %9, vcc\n"
"v_cndmask_b32 %6, %6, %9, vcc\n"
"v_cndmask_b32 %7, %7, %9, vcc\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_cmp_gt_u32_e64(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_cmp_gt_u32_e64 %8, %0, %9\n"
"v_cmp_gt_u32_e64 %8, %1, %9\n"
"v_cmp_gt_u32_e64 %8, %2, %9\n"
"v_cmp_gt_u32_e64 %8, %3, %9\n"
"v_cmp_gt_u32_e64 %8, %4, %9\n"
"v_cmp_gt_u32_e64 %8, %5, %9\n"
"v_cmp_gt_u32_e64 %8, %6, %9\n"
"v_cmp_gt_u32_e64 %8, %7, %9\n"
"v_cmp_gt_u32_e64 %8, %0, %9\n"
"v_cmp_gt_u32_e64 %8, %1, %9\n"
"v_cmp_gt_u32_e64 %8, %2, %9\n"
"v_cmp_gt_u32_e64 %8, %3, %9\n"
"v_cmp_gt_u32_e64 %8, %4, %9\n"
"v_cmp_gt_u32_e64 %8, %5, %9\n"
"v_cmp_gt_u32_e64 %8, %6, %9\n"
"v_cmp_gt_u32_e64 %8, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_add_co_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %9\n"
"v_add_co_u32 %1, vcc, %1, %9\n"
"v_add_co_u32 %2, vcc, %2, %9\n"
"v_add_co_u32 %3, vcc, %3, %9\n"
"v_add_co_u32 %4, vcc, %4, %9\n"
"v_add_co_u32 %5, vcc, %5, %9\n"
"v_add_co_u32 %6, vcc, %6, %9\n"
"v_add_co_u32 %7, vcc, %7, %9\n"
"v_add_co_u32 %0, vcc, %0, %9\n"
"v_add_co_u32 %1, vcc, %1, %9\n"
"v_add_co_u32 %2, vcc, %2, %9\n"
"v_add_co_u32 %3, vcc, %3, %9\n"
"v_add_co_u32 %4, vcc, %4, %9\n"
"v_add_co_u32 %5, vcc, %5, %9\n"
"v_add_co_u32 %6, vcc, %6, %9\n"
"v_add_co_u32 %7, vcc, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_lshlrev_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_lshlrev_b32 %0, 3, %0\n"
"v_lshlrev_b32 %1, 3, %1\n"
"v_lshlrev_b32 %2, 3, %2\n"
"v_lshlrev_b32 %3, 3, %3\n"
"v_lshlrev_b32 %4, 3, %4\n"
"v_lshlrev_b32 %5, 3, %5\n"
"v_lshlrev_b32 %6, 3, %6\n"
"v_lshlrev_b32 %7, 3, %7\n"
"v_lshlrev_b32 %0, 3, %0\n"
"v_lshlrev_b32 %1, 3, %1\n"
"v_lshlrev_b32 %2, 3, %2\n"
"v_lshlrev_b32 %3, 3, %3\n"
"v_lshlrev_b32 %4, 3, %4\n"
"v_lshlrev_b32 %5, 3, %5\n"
"v_lshlrev_b32 %6, 3, %6\n"
"v_lshlrev_b32 %7, 3, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_max_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_max_u16 %0, %0, %9\n"
"v_max_u16 %1, %1, %9\n"
"v_max_u16 %2, %2, %9\n"
"v_max_u16 %3, %3, %9\n"
"v_max_u16 %4, %4, %9\n"
"v_max_u16 %5, %5, %9\n"
"v_max_u16 %6, %6, %9\n"
"v_max_u16 %7, %7, %9\n"
"v_max_u16 %0, %0, %9\n"
"v_max_u16 %1, %1, %9\n"
"v_max_u16 %2, %2, %9\n"
"v_max_u16 %3, %3, %9\n"
"v_max_u16 %4, %4, %9\n"
"v_max_u16 %5, %5, %9\n"
"v_max_u16 %6, %6, %9\n"
"v_max_u16 %7, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_sub_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_sub_u16 %0, %0, %9\n"
"v_sub_u16 %1, %1, %9\n"
"v_sub_u16 %2, %2, %9\n"
"v_sub_u16 %3, %3, %9\n"
"v_sub_u16 %4, %4, %9\n"
"v_sub_u16 %5, %5, %9\n"
"v_sub_u16 %6, %6, %9\n"
"v_sub_u16 %7, %7, %9\n"
"v_sub_u16 %0, %0, %9\n"
"v_sub_u16 %1, %1, %9\n"
"v_sub_u16 %2, %2, %9\n"
"v_sub_u16 %3, %3, %9\n"
"v_sub_u16 %4, %4, %9\n"
"v_sub_u16 %5, %5, %9\n"
"v_sub_u16 %6, %6, %9\n"
"v_sub_u16 %7, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_mul_lo_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mul_lo_u16 %0, %0, %9\n"
"v_mul_lo_u16 %1, %1, %9\n"
"v_mul_lo_u16 %2, %2, %9\n"
"v_mul_lo_u16 %3, %3, %9\n"
"v_mul_lo_u16 %4, %4, %9\n"
"v_mul_lo_u16 %5, %5, %9\n"
"v_mul_lo_u16 %6, %6, %9\n"
"v_mul_lo_u16 %7, %7, %9\n"
"v_mul_lo_u16 %0, %0, %9\n"
"v_mul_lo_u16 %1, %1, %9\n"
"v_mul_lo_u16 %2, %2, %9\n"
"v_mul_lo_u16 %3, %3, %9\n"
"v_mul_lo_u16 %4, %4, %9\n"
"v_mul_lo_u16 %5, %5, %9\n"
"v_mul_lo_u16 %6, %6, %9\n"
"v_mul_lo_u16 %7, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_add_f16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_f16 %0, %0, %9\n"
"v_add_f16 %1, %1, %9\n"
"v_add_f16 %2, %2, %9\n"
"v_add_f16 %3, %3, %9\n"
"v_add_f16 %4, %4, %9\n"
"v_add_f16 %5, %5, %9\n"
"v_add_f16 %6, %6, %9\n"
"v_add_f16 %7, %7, %9\n"
"v_add_f16 %0, %0, %9\n"
"v_add_f16 %1, %1, %9\n"
"v_add_f16 %2, %2, %9\n"
"v_add_f16 %3, %3, %9\n"
"v_add_f16 %4, %4, %9\n"
"v_add_f16 %5, %5, %9\n"
"v_add_f16 %6, %6, %9\n"
"v_add_f16 %7, %7, %9\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_add_u16_sdwa(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_add_u16_sdwa %0, %0, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %1, %1, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %2, %2, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %3, %3, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %4, %4, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %5, %5, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %6, %6, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %7, %7, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %0, %0, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %1, %1, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %2, %2, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %3, %3, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %4, %4, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %5, %5, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %6, %6, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
"v_add_u16_sdwa %7, %7, %9 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_2\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_cvt_f32_ubyte1(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_cvt_f32_ubyte1 %0, %0\n"
"v_cvt_f32_ubyte1 %1, %1\n"
"v_cvt_f32_ubyte1 %2, %2\n"
"v_cvt_f32_ubyte1 %3, %3\n"
"v_cvt_f32_ubyte1 %4, %4\n"
"v_cvt_f32_ubyte1 %5, %5\n"
"v_cvt_f32_ubyte1 %6, %6\n"
"v_cvt_f32_ubyte1 %7, %7\n"
"v_cvt_f32_ubyte1 %0, %0\n"
"v_cvt_f32_ubyte1 %1, %1\n"
"v_cvt_f32_ubyte1 %2, %2\n"
"v_cvt_f32_ubyte1 %3, %3\n"
"v_cvt_f32_ubyte1 %4, %4\n"
"v_cvt_f32_ubyte1 %5, %5\n"
"v_cvt_f32_ubyte1 %6, %6\n"
"v_cvt_f32_ubyte1 %7, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_and_b32_literal(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_and_b32 %0, 0x00ff00ff, %0\n"
"v_and_b32 %1, 0x00ff00ff, %1\n"
"v_and_b32 %2, 0x00ff00ff, %2\n"
"v_and_b32 %3, 0x00ff00ff, %3\n"
"v_and_b32 %4, 0x00ff00ff, %4\n"
"v_and_b32 %5, 0x00ff00ff, %5\n"
"v_and_b32 %6, 0x00ff00ff, %6\n"
"v_and_b32 %7, 0x00ff00ff, %7\n"
"v_and_b32 %0, 0x00ff00ff, %0\n"
"v_and_b32 %1, 0x00ff00ff, %1\n"
"v_and_b32 %2, 0x00ff00ff, %2\n"
"v_and_b32 %3, 0x00ff00ff, %3\n"
"v_and_b32 %4, 0x00ff00ff, %4\n"
"v_and_b32 %5, 0x00ff00ff, %5\n"
"v_and_b32 %6, 0x00ff00ff, %6\n"
"v_and_b32 %7, 0x00ff00ff, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_mbcnt_lo_u32_b32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mbcnt_lo_u32_b32 %0, %10, %0\n"
"v_mbcnt_lo_u32_b32 %1, %10, %1\n"
"v_mbcnt_lo_u32_b32 %2, %10, %2\n"
"v_mbcnt_lo_u32_b32 %3, %10, %3\n"
"v_mbcnt_lo_u32_b32 %4, %10, %4\n"
"v_mbcnt_lo_u32_b32 %5, %10, %5\n"
"v_mbcnt_lo_u32_b32 %6, %10, %6\n"
"v_mbcnt_lo_u32_b32 %7, %10, %7\n"
"v_mbcnt_lo_u32_b32 %0, %10, %0\n"
"v_mbcnt_lo_u32_b32 %1, %10, %1\n"
"v_mbcnt_lo_u32_b32 %2, %10, %2\n"
"v_mbcnt_lo_u32_b32 %3, %10, %3\n"
"v_mbcnt_lo_u32_b32 %4, %10, %4\n"
"v_mbcnt_lo_u32_b32 %5, %10, %5\n"
"v_mbcnt_lo_u32_b32 %6, %10, %6\n"
"v_mbcnt_lo_u32_b32 %7, %10, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_lshrrev_b16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_lshrrev_b16 %0, 1, %0\n"
"v_lshrrev_b16 %1, 1, %1\n"
"v_lshrrev_b16 %2, 1, %2\n"
"v_lshrrev_b16 %3, 1, %3\n"
"v_lshrrev_b16 %4, 1, %4\n"
"v_lshrrev_b16 %5, 1, %5\n"
"v_lshrrev_b16 %6, 1, %6\n"
"v_lshrrev_b16 %7, 1, %7\n"
"v_lshrrev_b16 %0, 1, %0\n"
"v_lshrrev_b16 %1, 1, %1\n"
"v_lshrrev_b16 %2, 1, %2\n"
"v_lshrrev_b16 %3, 1, %3\n"
"v_lshrrev_b16 %4, 1, %4\n"
"v_lshrrev_b16 %5, 1, %5\n"
"v_lshrrev_b16 %6, 1, %6\n"
"v_lshrrev_b16 %7, 1, %7\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_sad_u16(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_sad_u16 %0, %0, %9, %10\n"
"v_sad_u16 %1, %1, %9, %10\n"
"v_sad_u16 %2, %2, %9, %10\n"
"v_sad_u16 %3, %3, %9, %10\n"
"v_sad_u16 %4, %4, %9, %10\n"
"v_sad_u16 %5, %5, %9, %10\n"
"v_sad_u16 %6, %6, %9, %10\n"
"v_sad_u16 %7, %7, %9, %10\n"
"v_sad_u16 %0, %0, %9, %10\n"
"v_sad_u16 %1, %1, %9, %10\n"
"v_sad_u16 %2, %2, %9, %10\n"
"v_sad_u16 %3, %3, %9, %10\n"
"v_sad_u16 %4, %4, %9, %10\n"
"v_sad_u16 %5, %5, %9, %10\n"
"v_sad_u16 %6, %6, %9, %10\n"
"v_sad_u16 %7, %7, %9, %10\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}
__global__ void __launch_bounds__(512) k_v_xad_u32(uint32_t* out, uint32_t seed) {
    uint32_t r[8];
    for (int q = 0; q < 8; ++q) r[q] = (threadIdx.x ^ seed) + q;
    const uint32_t k = seed | 1u, k2 = seed * 3u;
    unsigned long long sm = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_xad_u32 %0, %0, %9, %10\n"
"v_xad_u32 %1, %1, %9, %10\n"
"v_xad_u32 %2, %2, %9, %10\n"
"v_xad_u32 %3, %3, %9, %10\n"
"v_xad_u32 %4, %4, %9, %10\n"
"v_xad_u32 %5, %5, %9, %10\n"
"v_xad_u32 %6, %6, %9, %10\n"
"v_xad_u32 %7, %7, %9, %10\n"
"v_xad_u32 %0, %0, %9, %10\n"
"v_xad_u32 %1, %1, %9, %10\n"
"v_xad_u32 %2, %2, %9, %10\n"
"v_xad_u32 %3, %3, %9, %10\n"
"v_xad_u32 %4, %4, %9, %10\n"
"v_xad_u32 %5, %5, %9, %10\n"
"v_xad_u32 %6, %6, %9, %10\n"
"v_xad_u32 %7, %7, %9, %10\n"
                     : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+s"(sm)
                     : "v"(k), "v"(k2) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7] ^ (uint32_t)sm;
}

typedef void (*KFn)(uint32_t*, uint32_t);

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    uint32_t* out = nullptr;
    hipMalloc(&out, (size_t)ncu * 8 * 512 * 4 * 4);
    struct {
        const char* name;
        KFn fn;
    } ks[] = {{"v_add_u32", k_v_add_u32}, {"v_add_u32_e64", k_v_add_u32_e64}, {"v_sub_u32", k_v_sub_u32}, {"v_and_b32", k_v_and_b32}, {"v_or_b32", k_v_or_b32}, {"v_xor_b32", k_v_xor_b32}, {"v_lshrrev_b32", k_v_lshrrev_b32}, {"v_min_u32", k_v_min_u32}, {"v_max_i32", k_v_max_i32}, {"v_min_u16", k_v_min_u16}, {"v_mov_b32_dpp", k_v_mov_b32_dpp}, {"v_cndmask_b32", k_v_cndmask_b32}, {"v_add_f32", k_v_add_f32}, {"v_mul_f32", k_v_mul_f32}, {"v_fmac_f32", k_v_fmac_f32}, {"v_fma_f32", k_v_fma_f32}, {"v_pk_fma_f32", k_v_pk_fma_f32}, {"v_mul_u32_u24", k_v_mul_u32_u24}, {"v_mul_hi_u32_u24", k_v_mul_hi_u32_u24}, {"v_mad_u32_u24", k_v_mad_u32_u24}, {"v_mul_lo_u32", k_v_mul_lo_u32}, {"v_bfe_u32", k_v_bfe_u32}, {"v_bfi_b32", k_v_bfi_b32}, {"v_alignbyte_b32", k_v_alignbyte_b32}, {"v_perm_b32", k_v_perm_b32}, {"v_add3_u32", k_v_add3_u32}, {"v_lshl_or_b32", k_v_lshl_or_b32}, {"v_and_or_b32", k_v_and_or_b32}, {"v_min3_u32", k_v_min3_u32}, {"v_med3_u32", k_v_med3_u32}, {"v_sad_u8", k_v_sad_u8}, {"v_pk_min_u16", k_v_pk_min_u16}, {"v_pk_add_u16", k_v_pk_add_u16}, {"v_pk_add_f16", k_v_pk_add_f16}, {"v_pk_minimum3_f16", k_v_pk_minimum3_f16}, {"v_dot4_u32_u8", k_v_dot4_u32_u8}, {"v_dot2_u32_u16", k_v_dot2_u32_u16}, {"v_cvt_f32_u32", k_v_cvt_f32_u32}, {"mix_perm_add", k_mix_perm_add}, {"mix_pkmin_and", k_mix_pkmin_and}, {"mix_dot4_add", k_mix_dot4_add}, {"v_cndmask_b32_e64", k_v_cndmask_b32_e64}, {"v_cndmask_b32_vcc_set", k_v_cndmask_b32_vcc_set}, {"v_cmp_gt_u32_e64", k_v_cmp_gt_u32_e64}, {"v_add_co_u32", k_v_add_co_u32}, {"v_lshlrev_b32", k_v_lshlrev_b32}, {"v_max_u16", k_v_max_u16}, {"v_sub_u16", k_v_sub_u16}, {"v_mul_lo_u16", k_v_mul_lo_u16}, {"v_add_f16", k_v_add_f16}, {"v_add_u16_sdwa", k_v_add_u16_sdwa}, {"v_cvt_f32_ubyte1", k_v_cvt_f32_ubyte1}, {"v_and_b32_literal", k_v_and_b32_literal}, {"v_mbcnt_lo_u32_b32", k_v_mbcnt_lo_u32_b32}, {"v_lshrrev_b16", k_v_lshrrev_b16}, {"v_sad_u16", k_v_sad_u16}, {"v_xad_u32", k_v_xad_u32}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::printf("{\"cus\": %d, \"iter\": %d, \"rates\": {", ncu, ITER);
    bool firstK = true;
    for (auto& kk : ks) {
        std::printf("%s\"%s\": {", firstK ? "" : ", ", kk.name);
        firstK = false;
        // waves per SIMD w: 4 w waves per CU = one workgroup of 64*4*w threads per CU (w <= 2 per
        // 512-thread block; more blocks per CU for w > 2)
        const int wps[] = {1, 2, 4, 8};
        for (int wi = 0; wi < 4; ++wi) {
            const int w = wps[wi];
            const int threads = w <= 2 ? 256 * w : 512, blocks = w <= 2 ? ncu : ncu * (w / 2);
            hipLaunchKernelGGL(kk.fn, dim3(blocks), dim3(threads), 0, 0, out, 7u);
            hipDeviceSynchronize();
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(kk.fn, dim3(blocks), dim3(threads), 0, 0, out, 7u + rep);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            // wave-instructions per SIMD per ns
            const double winst = (double)blocks * threads / 64.0 * ITER * 16.0;
            const double perSimdNs = winst / (ncu * 4.0) / (best * 1e6);
            std::printf("%s\"w%d\": {\"ms\": %.4f, \"winst_per_simd_per_ns\": %.4f}", wi ? ", " : "", w, best,
                        perSimdNs);
        }
        std::printf("}");
    }
    std::printf("}}\n");
    hipFree(out);
    return 0;
}
