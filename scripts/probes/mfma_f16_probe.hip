// Probe (experiment harness): v_mfma_f32_16x16x32_f16 with f16-denormal byte inputs, against
// the exact integer product.  Prints the number of differing outputs per input encoding.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint4* a, const uint4* b, float4* d) {
    f16x8 A = __builtin_bit_cast(f16x8, a[threadIdx.x]), B = __builtin_bit_cast(f16x8, b[threadIdx.x]);
    f32x4 z = {0, 0, 0, 0};
    d[threadIdx.x] = __builtin_bit_cast(float4, __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, z, 0, 0, 0));
}
static uint16_t f16_of_int(int w) {  // positive integer < 2^11 * 2^k exactly representable
    if (!w) return 0;
    int e = 0;
    while ((w >> (e + 1)) != 0) ++e;
    return (uint16_t)(((e + 15) << 10) | (((w << 10) >> e) & 0x3FF));
}
static double f16_val(uint16_t h) {
    int e = (h >> 10) & 31, m = h & 1023;
    return e ? std::ldexp(1.0 + m / 1024.0, e - 15) : std::ldexp((double)m, -24);
}
int main() {
    uint16_t A[64 * 8], B[64 * 8];
    float D[64 * 4];
    uint4 *dA, *dB;
    float4* dD;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dB, sizeof(B));
    hipMalloc(&dD, sizeof(D));
    uint32_t s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
    for (int mode = 0; mode < 4; ++mode) {
        // mode 0: A = taps-like ints, B = bytes as denormals; 1: B = bytes as normals (int);
        // 2: one-hot K mapping check (A lane group h, j = 1 only at (h0, j0), B likewise); 3: A x256
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
                A[l * 8 + j] = f16_of_int(mode == 3 ? 256 * (int)(rnd() % 56) : (int)(rnd() % 56));
                const int bv = (int)(rnd() % 256);
                B[l * 8 + j] = mode == 1 ? f16_of_int(bv) : (uint16_t)bv;
            }
        hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
        hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
        hipMemcpy(D, dD, sizeof(D), hipMemcpyDeviceToHost);
        // reference: D[m][n] = sum_k A[m][k] B[k][n], lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]
        int bad = 0;
        double maxerr = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 4; ++i) {
                const int m = 4 * (l >> 4) + i, n = l & 15;
                double ref = 0;
                for (int kk = 0; kk < 32; ++kk) {
                    const int la = m + 16 * (kk >> 3), lb = n + 16 * (kk >> 3), jj = kk & 7;
                    ref += f16_val(A[la * 8 + jj]) * f16_val(B[lb * 8 + jj]);
                }
                const double got = D[l * 4 + i];
                if (got != ref) ++bad;
                maxerr = std::fmax(maxerr, std::fabs(got - ref) / (std::fabs(ref) + 1e-30));
                if (bad && bad < 3 && got != ref)
                    printf("  mode %d lane %d i %d: got %.10g ref %.10g (x2^24: %.3f vs %.3f)\n", mode, l, i, got, ref,
                           got * 16777216.0, ref * 16777216.0);
            }
        printf("mode %d: %d of 256 outputs differ, max rel err %g\n", mode, bad, maxerr);
    }
    return 0;
}
