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

}  // namespace cpu
}  // namespace dcnn_native
