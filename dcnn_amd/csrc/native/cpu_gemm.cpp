// Blocked, packed CPU GEMM (float and double) for the host compute backend.
//
// Reference: src/math/cpu/sgemm.cpp:485-653 (32x32 blocked AVX2 micro-kernels for NN/NT/TN, TT by
// transposed recompute, beta pre-scale) and src/math/cpu/dgemm.cpp; optional MKL path
// (include/utils/mkl_utils.hpp:18-143). Here one GotoBLAS-style driver covers every transpose
// combination: op(A) is packed into MR-row panels and op(B) into NR-column panels (the transpose is
// absorbed by the packing), an MR x NR register-blocked micro-kernel runs over a KC-deep panel pair,
// and (row block, column-panel group) tasks run on the native thread pool. The micro-kernel is
// picked at run time: AVX2+FMA (6x16 float / 6x8 double, 12 ymm accumulators) when the CPU has it,
// a portable scalar kernel otherwise — no -march flags, so the .so runs on any x86-64 host.
// Every output element is owned by one task and K is always walked in the same order: results
// are bit-identical across runs and thread counts.
#include "cpu_kernels.h"

#include <immintrin.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "threadpool.h"

namespace dcnn_native {
namespace cpu {

namespace {

template <typename T>
struct Blk;
template <>
struct Blk<float> {
  static constexpr int MR = 6, NR = 16, MC = 144, KC = 256, NC = 3072;
};
template <>
struct Blk<double> {
  static constexpr int MR = 6, NR = 8, MC = 96, KC = 256, NC = 1536;
};

bool has_avx2_fma() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}

// element (i, k) of op(A), (k, j) of op(B)
template <typename T>
inline T a_at(const T* A, long lda, bool ta, long i, long k) { return ta ? A[k * lda + i] : A[i * lda + k]; }
template <typename T>
inline T b_at(const T* B, long ldb, bool tb, long k, long j) { return tb ? B[j * ldb + k] : B[k * ldb + j]; }

// pack op(A)[i0:i0+mc, k0:k0+kc] into MR-row panels: dst[p][k][r], zero-padded rows
template <typename T>
void pack_a(const T* A, long lda, bool ta, long i0, long mc, long k0, long kc, T* dst) {
  constexpr int MR = Blk<T>::MR;
  for (long p = 0; p < mc; p += MR) {
    const int rows = (int)std::min<long>(MR, mc - p);
    T* d = dst + p * kc;
    if (!ta) {
      for (long k = 0; k < kc; ++k) {
        for (int r = 0; r < rows; ++r) d[k * MR + r] = A[(i0 + p + r) * lda + k0 + k];
        for (int r = rows; r < MR; ++r) d[k * MR + r] = T(0);
      }
    } else {
      for (long k = 0; k < kc; ++k) {
        const T* src = A + (k0 + k) * lda + i0 + p;
        for (int r = 0; r < rows; ++r) d[k * MR + r] = src[r];
        for (int r = rows; r < MR; ++r) d[k * MR + r] = T(0);
      }
    }
  }
}

// pack op(B)[k0:k0+kc, j0:j0+nc] into NR-column panels: dst[q][k][c], zero-padded columns
template <typename T>
void pack_b_panel(const T* B, long ldb, bool tb, long k0, long kc, long j, int cols, T* d) {
  constexpr int NR = Blk<T>::NR;
  if (!tb) {
    for (long k = 0; k < kc; ++k) {
      const T* src = B + (k0 + k) * ldb + j;
      for (int c = 0; c < cols; ++c) d[k * NR + c] = src[c];
      for (int c = cols; c < NR; ++c) d[k * NR + c] = T(0);
    }
  } else {
    for (long k = 0; k < kc; ++k) {
      for (int c = 0; c < cols; ++c) d[k * NR + c] = B[(j + c) * ldb + k0 + k];
      for (int c = cols; c < NR; ++c) d[k * NR + c] = T(0);
    }
  }
}

// ---- micro-kernels: Ctile[MR][NR] (ldc) += alpha * sum_k Ap[k][:] x Bp[k][:] ----
template <typename T>
void micro_scalar(long kc, const T* Ap, const T* Bp, T* C, long ldc, T alpha, int rows, int cols) {
  constexpr int MR = Blk<T>::MR, NR = Blk<T>::NR;
  T acc[MR][NR] = {};
  for (long k = 0; k < kc; ++k) {
    const T* a = Ap + k * MR;
    const T* b = Bp + k * NR;
    for (int r = 0; r < MR; ++r)
      for (int c = 0; c < NR; ++c) acc[r][c] += a[r] * b[c];
  }
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) C[r * ldc + c] += alpha * acc[r][c];
}

__attribute__((target("avx2,fma"))) void micro_avx2(long kc, const float* Ap, const float* Bp, float* C, long ldc,
                                                    float alpha, int rows, int cols) {
  __m256 c00 = _mm256_setzero_ps(), c01 = _mm256_setzero_ps(), c10 = _mm256_setzero_ps(), c11 = _mm256_setzero_ps();
  __m256 c20 = _mm256_setzero_ps(), c21 = _mm256_setzero_ps(), c30 = _mm256_setzero_ps(), c31 = _mm256_setzero_ps();
  __m256 c40 = _mm256_setzero_ps(), c41 = _mm256_setzero_ps(), c50 = _mm256_setzero_ps(), c51 = _mm256_setzero_ps();
  for (long k = 0; k < kc; ++k) {
    const __m256 b0 = _mm256_loadu_ps(Bp + k * 16), b1 = _mm256_loadu_ps(Bp + k * 16 + 8);
    const float* a = Ap + k * 6;
    __m256 a0 = _mm256_broadcast_ss(a + 0);
    c00 = _mm256_fmadd_ps(a0, b0, c00); c01 = _mm256_fmadd_ps(a0, b1, c01);
    a0 = _mm256_broadcast_ss(a + 1);
    c10 = _mm256_fmadd_ps(a0, b0, c10); c11 = _mm256_fmadd_ps(a0, b1, c11);
    a0 = _mm256_broadcast_ss(a + 2);
    c20 = _mm256_fmadd_ps(a0, b0, c20); c21 = _mm256_fmadd_ps(a0, b1, c21);
    a0 = _mm256_broadcast_ss(a + 3);
    c30 = _mm256_fmadd_ps(a0, b0, c30); c31 = _mm256_fmadd_ps(a0, b1, c31);
    a0 = _mm256_broadcast_ss(a + 4);
    c40 = _mm256_fmadd_ps(a0, b0, c40); c41 = _mm256_fmadd_ps(a0, b1, c41);
    a0 = _mm256_broadcast_ss(a + 5);
    c50 = _mm256_fmadd_ps(a0, b0, c50); c51 = _mm256_fmadd_ps(a0, b1, c51);
  }
  alignas(32) float t[6][16];
  const __m256 al = _mm256_set1_ps(alpha);
  _mm256_store_ps(t[0], _mm256_mul_ps(al, c00)); _mm256_store_ps(t[0] + 8, _mm256_mul_ps(al, c01));
  _mm256_store_ps(t[1], _mm256_mul_ps(al, c10)); _mm256_store_ps(t[1] + 8, _mm256_mul_ps(al, c11));
  _mm256_store_ps(t[2], _mm256_mul_ps(al, c20)); _mm256_store_ps(t[2] + 8, _mm256_mul_ps(al, c21));
  _mm256_store_ps(t[3], _mm256_mul_ps(al, c30)); _mm256_store_ps(t[3] + 8, _mm256_mul_ps(al, c31));
  _mm256_store_ps(t[4], _mm256_mul_ps(al, c40)); _mm256_store_ps(t[4] + 8, _mm256_mul_ps(al, c41));
  _mm256_store_ps(t[5], _mm256_mul_ps(al, c50)); _mm256_store_ps(t[5] + 8, _mm256_mul_ps(al, c51));
  if (cols == 16) {
    for (int r = 0; r < rows; ++r) {
      float* cr = C + r * ldc;
      _mm256_storeu_ps(cr, _mm256_add_ps(_mm256_loadu_ps(cr), _mm256_load_ps(t[r])));
      _mm256_storeu_ps(cr + 8, _mm256_add_ps(_mm256_loadu_ps(cr + 8), _mm256_load_ps(t[r] + 8)));
    }
  } else {
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) C[r * ldc + c] += t[r][c];
  }
}

__attribute__((target("avx2,fma"))) void micro_avx2(long kc, const double* Ap, const double* Bp, double* C, long ldc,
                                                    double alpha, int rows, int cols) {
  __m256d c00 = _mm256_setzero_pd(), c01 = _mm256_setzero_pd(), c10 = _mm256_setzero_pd(), c11 = _mm256_setzero_pd();
  __m256d c20 = _mm256_setzero_pd(), c21 = _mm256_setzero_pd(), c30 = _mm256_setzero_pd(), c31 = _mm256_setzero_pd();
  __m256d c40 = _mm256_setzero_pd(), c41 = _mm256_setzero_pd(), c50 = _mm256_setzero_pd(), c51 = _mm256_setzero_pd();
  for (long k = 0; k < kc; ++k) {
    const __m256d b0 = _mm256_loadu_pd(Bp + k * 8), b1 = _mm256_loadu_pd(Bp + k * 8 + 4);
    const double* a = Ap + k * 6;
    __m256d a0 = _mm256_broadcast_sd(a + 0);
    c00 = _mm256_fmadd_pd(a0, b0, c00); c01 = _mm256_fmadd_pd(a0, b1, c01);
    a0 = _mm256_broadcast_sd(a + 1);
    c10 = _mm256_fmadd_pd(a0, b0, c10); c11 = _mm256_fmadd_pd(a0, b1, c11);
    a0 = _mm256_broadcast_sd(a + 2);
    c20 = _mm256_fmadd_pd(a0, b0, c20); c21 = _mm256_fmadd_pd(a0, b1, c21);
    a0 = _mm256_broadcast_sd(a + 3);
    c30 = _mm256_fmadd_pd(a0, b0, c30); c31 = _mm256_fmadd_pd(a0, b1, c31);
    a0 = _mm256_broadcast_sd(a + 4);
    c40 = _mm256_fmadd_pd(a0, b0, c40); c41 = _mm256_fmadd_pd(a0, b1, c41);
    a0 = _mm256_broadcast_sd(a + 5);
    c50 = _mm256_fmadd_pd(a0, b0, c50); c51 = _mm256_fmadd_pd(a0, b1, c51);
  }
  alignas(32) double t[6][8];
  const __m256d al = _mm256_set1_pd(alpha);
  _mm256_store_pd(t[0], _mm256_mul_pd(al, c00)); _mm256_store_pd(t[0] + 4, _mm256_mul_pd(al, c01));
  _mm256_store_pd(t[1], _mm256_mul_pd(al, c10)); _mm256_store_pd(t[1] + 4, _mm256_mul_pd(al, c11));
  _mm256_store_pd(t[2], _mm256_mul_pd(al, c20)); _mm256_store_pd(t[2] + 4, _mm256_mul_pd(al, c21));
  _mm256_store_pd(t[3], _mm256_mul_pd(al, c30)); _mm256_store_pd(t[3] + 4, _mm256_mul_pd(al, c31));
  _mm256_store_pd(t[4], _mm256_mul_pd(al, c40)); _mm256_store_pd(t[4] + 4, _mm256_mul_pd(al, c41));
  _mm256_store_pd(t[5], _mm256_mul_pd(al, c50)); _mm256_store_pd(t[5] + 4, _mm256_mul_pd(al, c51));
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) C[r * ldc + c] += t[r][c];
}

template <typename T>
void scale_c(T* C, long M, long N, long ldc, T beta) {
  if (beta == T(1)) return;
  parallel_for(0, M, std::max(1L, 16384 / std::max(1L, N)), [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) {
      T* c = C + i * ldc;
      if (beta == T(0))
        std::fill(c, c + N, T(0));
      else
        for (long j = 0; j < N; ++j) c[j] *= beta;
    }
  });
}

template <typename T>
void gemm_impl(bool ta, bool tb, long M, long N, long K, T alpha, const T* A, long lda, const T* B, long ldb, T beta,
               T* C, long ldc) {
  using Bk = Blk<T>;
  constexpr int MR = Bk::MR, NR = Bk::NR;
  scale_c(C, M, N, ldc, beta);
  if (M <= 0 || N <= 0 || K <= 0 || alpha == T(0)) return;
  const bool avx = has_avx2_fma();
  std::vector<T> bpack;
  for (long jc = 0; jc < N; jc += Bk::NC) {
    const long nc = std::min<long>(Bk::NC, N - jc);
    const long npan = (nc + NR - 1) / NR;
    for (long pc = 0; pc < K; pc += Bk::KC) {
      const long kc = std::min<long>(Bk::KC, K - pc);
      bpack.resize((size_t)npan * NR * kc);
      T* bp = bpack.data();
      parallel_for(0, npan, std::max(1L, 4096 / kc), [&](long lo, long hi) {
        for (long q = lo; q < hi; ++q)
          pack_b_panel(B, ldb, tb, pc, kc, jc + q * NR, (int)std::min<long>(NR, nc - q * NR), bp + q * kc * NR);
      });
      // tasks: (row block of MC) x (group of column panels); more groups when rows are few
      const long mblocks = (M + Bk::MC - 1) / Bk::MC;
      const long want = (long)get_num_threads() * 2;
      const long groups = std::max(1L, std::min(npan, (want + mblocks - 1) / mblocks));
      ThreadPool::instance().run(mblocks * groups, [&](long task) {
        const long ib = task / groups, g = task % groups;
        const long i0 = ib * Bk::MC, mc = std::min<long>(Bk::MC, M - i0);
        const long q0 = g * npan / groups, q1 = (g + 1) * npan / groups;
        thread_local std::vector<T> apack;
        apack.resize((size_t)((mc + MR - 1) / MR) * MR * kc);
        pack_a(A, lda, ta, i0, mc, pc, kc, apack.data());
        for (long q = q0; q < q1; ++q) {
          const int cols = (int)std::min<long>(NR, nc - q * NR);
          const T* bq = bp + q * kc * NR;
          for (long p = 0; p < mc; p += MR) {
            const int rows = (int)std::min<long>(MR, mc - p);
            T* ct = C + (i0 + p) * ldc + jc + q * NR;
            if (avx)
              micro_avx2(kc, apack.data() + p * kc, bq, ct, ldc, alpha, rows, cols);
            else
              micro_scalar<T>(kc, apack.data() + p * kc, bq, ct, ldc, alpha, rows, cols);
          }
        }
      });
    }
  }
}

}  // namespace

void gemm(bool ta, bool tb, long M, long N, long K, float alpha, const float* A, long lda, const float* B, long ldb,
          float beta, float* C, long ldc) {
  gemm_impl<float>(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}
void gemm(bool ta, bool tb, long M, long N, long K, double alpha, const double* A, long lda, const double* B, long ldb,
          double beta, double* C, long ldc) {
  gemm_impl<double>(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}
bool gemm_uses_avx2() { return has_avx2_fma(); }

}  // namespace cpu
}  // namespace dcnn_native
