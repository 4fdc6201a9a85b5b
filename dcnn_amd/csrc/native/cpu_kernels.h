// Native CPU compute backend (host side of the framework; the GPU side is csrc/kernels/*.hip).
//
// Reference: src/math/cpu/sgemm.cpp / dgemm.cpp (blocked GEMM), src/ops/cpu/skernels.cpp /
// dkernels.cpp (elementwise + reductions), include/tensor/cpu/tensor_ops.hpp (im2col/col2im/pad),
// src/nn/layers_impl/cpu/*_ops.cpp (conv, batchnorm, pooling). Every routine is templated on
// float/double, runs on the native ThreadPool, and is deterministic (fixed chunking, fixed
// reduction order). Layouts are NCHW contiguous, as in the reference's CPU path.
#pragma once
#include <cstdint>

namespace dcnn_native {
namespace cpu {

// C[M,N] = alpha * op(A)[M,K] @ op(B)[K,N] + beta * C   (row-major; ta/tb transpose A/B)
void gemm(bool ta, bool tb, long M, long N, long K, float alpha, const float* A, long lda, const float* B, long ldb,
          float beta, float* C, long ldc);
void gemm(bool ta, bool tb, long M, long N, long K, double alpha, const double* A, long lda, const double* B, long ldb,
          double beta, double* C, long ldc);
bool gemm_uses_avx2();
bool gemm_uses_avx512();

template <typename T> void elementwise(int mode, int op, const T* a, const T* b, T* c, long n, double s0, double s1);
template <typename T> double reduce(int op, const T* a, const T* b, long n);
template <typename T> void fill_random(T* out, long n, uint64_t seed, double a, double b, int normal);
template <typename T> void transpose2d(const T* in, T* out, long batch, long rows, long cols);
template <typename T> void swap01(const T* in, T* out, long A, long B, long HW);
template <typename T> void pad2d(const T* x, T* y, long NC, int H, int W, int ph, int pw, double value);
template <typename T> void crop2d(const T* x, T* y, long NC, int H, int W, int top, int left, int OH, int OW);
template <typename T>
void im2col(const T* x, T* col, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW);
template <typename T>
void col2im(const T* col, T* x, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW);
template <typename T>
void conv2d_fwd(const T* x, const T* w, const T* bias, T* y, int N, int C, int H, int W, int Co, int KH, int KW, int SH,
                int SW, int PH, int PW);
template <typename T>
void conv2d_bwd(const T* x, const T* w, const T* dy, T* dx, T* dw, T* db, int N, int C, int H, int W, int Co, int KH,
                int KW, int SH, int SW, int PH, int PW);
template <typename T> void dense_fwd(const T* x, const T* w, const T* bias, T* y, long N, long In, long Out);
template <typename T>
void dense_bwd(const T* x, const T* w, const T* dy, T* dx, T* dw, T* db, long N, long In, long Out);
template <typename T>
void batchnorm_fwd(const T* x, T* y, long N, long C, long HW, const T* gamma, const T* beta, double eps, int training,
                   T* running_mean, T* running_var, double momentum, T* save_mean, T* save_istd, int relu,
                   const T* residual);
template <typename T>
void batchnorm_bwd(const T* x, const T* dy, const T* yout, const T* mean, const T* istd, const T* gamma, T* dx,
                   T* dgamma, T* dbeta, T* masked_out, long N, long C, long HW, int training);
template <typename T>
void groupnorm_fwd(const T* x, T* y, long N, long C, long HW, long G, const T* gamma, const T* beta, double eps,
                   T* save_mean, T* save_istd);
template <typename T>
void groupnorm_bwd(const T* x, const T* dy, const T* mean, const T* istd, const T* gamma, T* dx, T* dgamma, T* dbeta,
                   long N, long C, long HW, long G);
template <typename T>
void maxpool_fwd(const T* x, T* y, int32_t* idx, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW);
template <typename T> void maxpool_bwd(const T* dy, const int32_t* idx, T* dx, long NC, int H, int W, int OH, int OW);
template <typename T>
void avgpool_fwd(const T* x, T* y, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW);
template <typename T>
void avgpool_bwd(const T* dy, T* dx, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW);
template <typename T> void act_fwd(int type, const T* x, T* y, long n, double alpha);
template <typename T> void act_bwd(int type, const T* x, const T* dy, T* dx, long n, double alpha);
template <typename T> void softmax_channels(const T* x, T* y, long N, long C, long HW);
template <typename T> void softmax_channels_bwd(const T* y, const T* dy, T* dx, long N, long C, long HW);
template <typename T>
double loss_fused(int kind, const T* pred, const T* target, const int64_t* labels, T* grad, long N, long C,
                  double param, long* correct);
template <typename T> void sgd_step(T* p, const T* g, T* vel, long n, double lr, double momentum);
template <typename T>
void adam_step(T* p, const T* g, T* m, T* v, long n, double lr, double b1, double b2, double eps, double bc1,
               double bc2, double wd, int decoupled);

}  // namespace cpu
}  // namespace dcnn_native
