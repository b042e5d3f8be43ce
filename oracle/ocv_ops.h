/*
 * ocv_ops.h — TEST INFRASTRUCTURE ONLY.  OpenCV 2.4 cv::Mat arithmetic the matchers use on
 * 3-vectors, restated (OpenCV is not installed here: parity unpinned against a real build;
 * DESIGN.md §FP policy states the semantics).  Compiled WITHOUT contraction (ocv_ops.cpp,
 * -ffp-contract=off): a distro OpenCV 2.4 targets baseline x86-64 and has no FMA.
 */
#ifndef OCV_OPS_H
#define OCV_OPS_H
namespace ocv {
// A(3x3, CV_32F) * x(3x1) + t  ==  MatExpr A*x+t -> gemm(A, x, 1, t, 1, D), flags 0: the
// 2 <= len <= 4 fast path: float t_i = a_i0*x0 + a_i1*x1 + a_i2*x2 (left to right), then
// d_i = (float)((double)t_i * alpha + (double)c_i * beta) with alpha = beta = 1.
void gemm3_add(const float* A, const float* x, const float* t, float* out);
// a - b element-wise (cv::subtract, float).
void sub3(const float* a, const float* b, float* out);
// cv::norm(v, NORM_L2) of a continuous 3x1 CV_32F: sqrt of normL2Sqr<float, double>
// (s = 0; s += (double)v_i * v_i, i = 0..2), returned as double.
double norm3(const float* v);
// Mat::dot of two continuous 3x1 CV_32F: dotProd_<float> (r = 0; r += (double)a_i * b_i).
double dot3(const float* a, const float* b);
}  // namespace ocv
#endif
