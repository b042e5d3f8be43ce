// TEST INFRASTRUCTURE ONLY — see ocv_ops.h.  Build with -ffp-contract=off.
#include "ocv_ops.h"

#include <cmath>

namespace ocv {
void gemm3_add(const float* A, const float* x, const float* t, float* out) {
    const double alpha = 1.0, beta = 1.0;
    for (int i = 0; i < 3; ++i) {
        const float ti = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
        out[i] = (float)(ti * alpha + t[i] * beta);
    }
}
void sub3(const float* a, const float* b, float* out) {
    for (int i = 0; i < 3; ++i) out[i] = a[i] - b[i];
}
double norm3(const float* v) {
    double s = 0;
    for (int i = 0; i < 3; ++i) {
        const double e = v[i];
        s += e * e;
    }
    return std::sqrt(s);
}
double dot3(const float* a, const float* b) {
    double r = 0;
    for (int i = 0; i < 3; ++i) r += (double)a[i] * b[i];
    return r;
}
}  // namespace ocv
