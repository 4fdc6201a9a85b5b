// Blocked, packed CPU GEMM (float and double) for the host compute backend.
//
// Reference: src/math/cpu/sgemm.cpp:485-653 (32x32 blocked AVX2 micro-kernels for NN/NT/TN, TT by
// transposed recompute, beta pre-scale) and src/math/cpu/dgemm.cpp; optional MKL path
// (include/utils/mkl_utils.hpp:18-143). Here one GotoBLAS-style driver covers every transpose
// combination: op(A) is packed into MR-row panels and op(B) into NR-column panels (the transpose is
// absorbed by the packing), an MR x NR register-blocked micro-kernel runs over a KC-deep panel pair,
// and (row block, column-panel group) tasks run on the native thread pool. The micro-kernel family
// is picked at run time from the CPU's features — AVX-512 (6x32 float / 6x16 double, 12 zmm
// accumulators), AVX2+FMA (6x16 / 6x8, 12 ymm accumulators) or portable scalar — with no -march
// flags, so the .so runs on any x86-64 host.
//
// Shapes with a small output and a long reduction (a convolution's weight gradient: Co x K outputs
// summed over N*OH*OW) are split along K into a FIXED number of slices (independent of the thread
// count), each reduced into its own partial, and the partials are summed in slice order. Every output
// element is owned by one task and K is always walked in the same order: results are bit-identical
// across runs and thread counts.
#include <immintrin.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "cpu_kernels.h"
#include "threadpool.h"

namespace dcnn_native {
namespace cpu {

namespace {

bool has_avx2_fma() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}
bool has_avx512() {
  static const bool ok = __builtin_cpu_supports("avx512f");
  return ok;
}

// ---- micro-kernels: Ctile[rows][cols] (ldc) += alpha * sum_k Ap[k][0:MR] x Bp[k][0:NR] ----
template <typename T, int MR, int NR>
void micro_scalar(long kc, const T* Ap, const T* Bp, T* C, long ldc, T alpha, int rows, int cols) {
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

template <typename T, int MR, int NR>
inline void store_tile(const T (&t)[MR][NR], T* C, long ldc, int rows, int cols) {
  for (int r = 0; r < rows; ++r) {
    T* cr = C + r * ldc;
    for (int c = 0; c < cols; ++c) cr[c] += t[r][c];
  }
}

// AVX2: 6 x 16 float (two ymm per row)
__attribute__((target("avx2,fma"))) void micro_avx2_f(long kc, const float* Ap, const float* Bp, float* C, long ldc,
                                                      float alpha, int rows, int cols) {
  __m256 c[6][2];
  for (int r = 0; r < 6; ++r) c[r][0] = c[r][1] = _mm256_setzero_ps();
  for (long k = 0; k < kc; ++k) {
    const __m256 b0 = _mm256_loadu_ps(Bp + k * 16), b1 = _mm256_loadu_ps(Bp + k * 16 + 8);
    const float* a = Ap + k * 6;
#pragma GCC unroll 6
    for (int r = 0; r < 6; ++r) {
      const __m256 av = _mm256_broadcast_ss(a + r);
      c[r][0] = _mm256_fmadd_ps(av, b0, c[r][0]);
      c[r][1] = _mm256_fmadd_ps(av, b1, c[r][1]);
    }
  }
  const __m256 al = _mm256_set1_ps(alpha);
  if (rows == 6 && cols == 16) {
    for (int r = 0; r < 6; ++r) {
      float* cr = C + r * ldc;
      _mm256_storeu_ps(cr, _mm256_fmadd_ps(al, c[r][0], _mm256_loadu_ps(cr)));
      _mm256_storeu_ps(cr + 8, _mm256_fmadd_ps(al, c[r][1], _mm256_loadu_ps(cr + 8)));
    }
    return;
  }
  alignas(32) float t[6][16];
  for (int r = 0; r < 6; ++r) {
    _mm256_store_ps(t[r], _mm256_mul_ps(al, c[r][0]));
    _mm256_store_ps(t[r] + 8, _mm256_mul_ps(al, c[r][1]));
  }
  store_tile<float, 6, 16>(t, C, ldc, rows, cols);
}

// AVX2: 6 x 8 double
__attribute__((target("avx2,fma"))) void micro_avx2_d(long kc, const double* Ap, const double* Bp, double* C, long ldc,
                                                      double alpha, int rows, int cols) {
  __m256d c[6][2];
  for (int r = 0; r < 6; ++r) c[r][0] = c[r][1] = _mm256_setzero_pd();
  for (long k = 0; k < kc; ++k) {
    const __m256d b0 = _mm256_loadu_pd(Bp + k * 8), b1 = _mm256_loadu_pd(Bp + k * 8 + 4);
    const double* a = Ap + k * 6;
#pragma GCC unroll 6
    for (int r = 0; r < 6; ++r) {
      const __m256d av = _mm256_broadcast_sd(a + r);
      c[r][0] = _mm256_fmadd_pd(av, b0, c[r][0]);
      c[r][1] = _mm256_fmadd_pd(av, b1, c[r][1]);
    }
  }
  alignas(32) double t[6][8];
  const __m256d al = _mm256_set1_pd(alpha);
  for (int r = 0; r < 6; ++r) {
    _mm256_store_pd(t[r], _mm256_mul_pd(al, c[r][0]));
    _mm256_store_pd(t[r] + 4, _mm256_mul_pd(al, c[r][1]));
  }
  store_tile<double, 6, 8>(t, C, ldc, rows, cols);
}

// AVX-512: 6 x 32 float (two zmm per row)
__attribute__((target("avx512f"))) void micro_avx512_f(long kc, const float* Ap, const float* Bp, float* C, long ldc,
                                                       float alpha, int rows, int cols) {
  __m512 c[6][2];
  for (int r = 0; r < 6; ++r) c[r][0] = c[r][1] = _mm512_setzero_ps();
  for (long k = 0; k < kc; ++k) {
    const __m512 b0 = _mm512_loadu_ps(Bp + k * 32), b1 = _mm512_loadu_ps(Bp + k * 32 + 16);
    const float* a = Ap + k * 6;
#pragma GCC unroll 6
    for (int r = 0; r < 6; ++r) {
      const __m512 av = _mm512_set1_ps(a[r]);
      c[r][0] = _mm512_fmadd_ps(av, b0, c[r][0]);
      c[r][1] = _mm512_fmadd_ps(av, b1, c[r][1]);
    }
  }
  const __m512 al = _mm512_set1_ps(alpha);
  if (rows == 6 && cols == 32) {
    for (int r = 0; r < 6; ++r) {
      float* cr = C + r * ldc;
      _mm512_storeu_ps(cr, _mm512_fmadd_ps(al, c[r][0], _mm512_loadu_ps(cr)));
      _mm512_storeu_ps(cr + 16, _mm512_fmadd_ps(al, c[r][1], _mm512_loadu_ps(cr + 16)));
    }
    return;
  }
  alignas(64) float t[6][32];
  for (int r = 0; r < 6; ++r) {
    _mm512_store_ps(t[r], _mm512_mul_ps(al, c[r][0]));
    _mm512_store_ps(t[r] + 16, _mm512_mul_ps(al, c[r][1]));
  }
  store_tile<float, 6, 32>(t, C, ldc, rows, cols);
}

// AVX-512: 6 x 16 double
__attribute__((target("avx512f"))) void micro_avx512_d(long kc, const double* Ap, const double* Bp, double* C,
                                                       long ldc, double alpha, int rows, int cols) {
  __m512d c[6][2];
  for (int r = 0; r < 6; ++r) c[r][0] = c[r][1] = _mm512_setzero_pd();
  for (long k = 0; k < kc; ++k) {
    const __m512d b0 = _mm512_loadu_pd(Bp + k * 16), b1 = _mm512_loadu_pd(Bp + k * 16 + 8);
    const double* a = Ap + k * 6;
#pragma GCC unroll 6
    for (int r = 0; r < 6; ++r) {
      const __m512d av = _mm512_set1_pd(a[r]);
      c[r][0] = _mm512_fmadd_pd(av, b0, c[r][0]);
      c[r][1] = _mm512_fmadd_pd(av, b1, c[r][1]);
    }
  }
  alignas(64) double t[6][16];
  const __m512d al = _mm512_set1_pd(alpha);
  for (int r = 0; r < 6; ++r) {
    _mm512_store_pd(t[r], _mm512_mul_pd(al, c[r][0]));
    _mm512_store_pd(t[r] + 8, _mm512_mul_pd(al, c[r][1]));
  }
  store_tile<double, 6, 16>(t, C, ldc, rows, cols);
}

// ---- kernel families: blocking + micro-kernel ----
template <typename T, int MR_, int NR_, int MC_, int KC_, int NC_>
struct Family {
  static constexpr int MR = MR_, NR = NR_, MC = MC_, KC = KC_, NC = NC_;
  using Micro = void (*)(long, const T*, const T*, T*, long, T, int, int);
  Micro micro;
};

// pack op(A)[i0:i0+mc, k0:k0+kc] into MR-row panels: dst[p][k][r], zero-padded rows
template <typename T, int MR>
void pack_a(const T* A, long lda, bool ta, long i0, long mc, long k0, long kc, T* dst) {
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

// pack op(B)[k0:k0+kc, j:j+cols] into one NR-column panel: d[k][c], zero-padded columns
template <typename T, int NR>
void pack_b_panel(const T* B, long ldb, bool tb, long k0, long kc, long j, int cols, T* d) {
  if (!tb) {
    for (long k = 0; k < kc; ++k) {
      const T* src = B + (k0 + k) * ldb + j;
      for (int c = 0; c < cols; ++c) d[k * NR + c] = src[c];
      for (int c = cols; c < NR; ++c) d[k * NR + c] = T(0);
    }
  } else {
    for (int c = 0; c < cols; ++c) {
      const T* src = B + (j + c) * ldb + k0;
      for (long k = 0; k < kc; ++k) d[k * NR + c] = src[k];
    }
    for (long k = 0; k < kc; ++k)
      for (int c = cols; c < NR; ++c) d[k * NR + c] = T(0);
  }
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

// C += alpha * op(A) op(B) over k in [k0, k1). `serial` runs everything on the calling thread.
template <typename T, typename F>
void gemm_accumulate(const F& fam, bool ta, bool tb, long M, long N, long k0, long k1, T alpha, const T* A, long lda,
                     const T* B, long ldb, T* C, long ldc, bool serial) {
  constexpr int MR = F::MR, NR = F::NR, MC = F::MC, KC = F::KC, NC = F::NC;
  std::vector<T> bpack, apack;
  if (!serial && M <= MC) {
    // one row block (small M, e.g. a conv's output channels over the whole batch's pixels): no
    // packed B panel is reused by another row block, so there is nothing to gain from NC
    // blocking or a shared B pack. A (M x kc) is packed once; ONE parallel region per K panel,
    // each task packing its own B panels into a thread-local buffer right before using them
    // (the NC-blocked schedule took two pool dispatches per 4096 columns: 40x slower on
    // 8 x 36864 x 25).
    // K panels of up to 4 x KC: one pool dispatch per panel is the dominant cost at these sizes
    // (an A panel of MC x 4KC and a 4KC x NR B panel still fit the L2)
    for (long pc = k0; pc < k1; pc += 4 * KC) {
      const long kc = std::min<long>(4 * KC, k1 - pc);
      apack.resize((size_t)((M + MR - 1) / MR) * MR * kc);
      pack_a<T, MR>(A, lda, ta, 0, M, pc, kc, apack.data());
      const long npan = (N + NR - 1) / NR;
      const long tasks = std::min<long>(npan, (long)get_num_threads() * 4);
      ThreadPool::instance().run(tasks, [&](long task) {
        thread_local std::vector<T> bl;
        bl.resize((size_t)kc * NR);
        const long q0 = task * npan / tasks, q1 = (task + 1) * npan / tasks;
        for (long q = q0; q < q1; ++q) {
          const int cols = (int)std::min<long>(NR, N - q * NR);
          pack_b_panel<T, NR>(B, ldb, tb, pc, kc, q * NR, cols, bl.data());
          for (long p = 0; p < M; p += MR) {
            const int rows = (int)std::min<long>(MR, M - p);
            fam.micro(kc, apack.data() + p * kc, bl.data(), C + p * ldc + q * NR, ldc, alpha, rows, cols);
          }
        }
      });
    }
    return;
  }
  for (long jc = 0; jc < N; jc += NC) {
    const long nc = std::min<long>(NC, N - jc);
    const long npan = (nc + NR - 1) / NR;
    for (long pc = k0; pc < k1; pc += KC) {
      const long kc = std::min<long>(KC, k1 - pc);
      bpack.resize((size_t)npan * NR * kc);
      const long mblocks = (M + MC - 1) / MC;
      const long arows = mblocks * MC;
      apack.resize((size_t)((arows + MR - 1) / MR) * MR * kc);
      T* bp = bpack.data();
      T* ap = apack.data();
      // pack every B panel and every A row block once (one parallel region)
      auto pack = [&](long t) {
        if (t < npan) {
          pack_b_panel<T, NR>(B, ldb, tb, pc, kc, jc + t * NR, (int)std::min<long>(NR, nc - t * NR), bp + t * kc * NR);
        } else {
          const long ib = t - npan, i0 = ib * MC;
          pack_a<T, MR>(A, lda, ta, i0, std::min<long>(MC, M - i0), pc, kc, ap + i0 * kc);
        }
      };
      if (serial) {
        for (long t = 0; t < npan + mblocks; ++t) pack(t);
      } else {
        ThreadPool::instance().run(npan + mblocks, pack);
      }
      // tasks: (row block) x (group of column panels); more groups when row blocks are few
      const long want = serial ? 1 : (long)get_num_threads() * 2;
      const long groups = std::max(1L, std::min(npan, (want + mblocks - 1) / mblocks));
      auto compute = [&](long task) {
        const long ib = task / groups, g = task % groups;
        const long i0 = ib * MC, mc = std::min<long>(MC, M - i0);
        const long q0 = g * npan / groups, q1 = (g + 1) * npan / groups;
        const T* aps = ap + i0 * kc;
        for (long q = q0; q < q1; ++q) {
          const int cols = (int)std::min<long>(NR, nc - q * NR);
          const T* bq = bp + q * kc * NR;
          for (long p = 0; p < mc; p += MR) {
            const int rows = (int)std::min<long>(MR, mc - p);
            fam.micro(kc, aps + p * kc, bq, C + (i0 + p) * ldc + jc + q * NR, ldc, alpha, rows, cols);
          }
        }
      };
      if (serial) {
        for (long t = 0; t < mblocks * groups; ++t) compute(t);
      } else {
        ThreadPool::instance().run(mblocks * groups, compute);
      }
    }
  }
}

template <typename T, typename F>
void gemm_impl(const F& fam, bool ta, bool tb, long M, long N, long K, T alpha, const T* A, long lda, const T* B,
               long ldb, T beta, T* C, long ldc) {
  scale_c(C, M, N, ldc, beta);
  if (M <= 0 || N <= 0 || K <= 0 || alpha == T(0)) return;
  // small output, long reduction: fixed K slices into private partials, summed in slice order
  const long slices = std::min<long>(16, K / (4L * F::KC));
  if (slices >= 2 && M * N <= 96L * 1024) {  // (inside a parallel region the slices run serially)
    // the calling thread's reusable partials buffer (no per-call allocation / page faults); the
    // pool tasks use it through this pointer (a thread_local named inside the lambda would be
    // each worker's own instance)
    thread_local std::vector<T> part_tl;
    part_tl.assign((size_t)slices * M * N, T(0));
    T* const part_p = part_tl.data();
    ThreadPool::instance().run(slices, [&](long s) {
      const long k0 = s * K / slices, k1 = (s + 1) * K / slices;
      gemm_accumulate(fam, ta, tb, M, N, k0, k1, alpha, A, lda, B, ldb, part_p + s * M * N, N, true);
    });
    parallel_for(0, M, std::max(1L, 4096 / N), [&](long lo, long hi) {
      for (long i = lo; i < hi; ++i)
        for (long s = 0; s < slices; ++s) {
          const T* pr = part_p + (s * M + i) * N;
          T* cr = C + i * ldc;
          for (long j = 0; j < N; ++j) cr[j] += pr[j];
        }
    });
    return;
  }
  gemm_accumulate(fam, ta, tb, M, N, 0, K, alpha, A, lda, B, ldb, C, ldc, in_parallel_region());
}

using F512 = Family<float, 6, 32, 192, 256, 4096>;
using D512 = Family<double, 6, 16, 96, 256, 2048>;
using F256 = Family<float, 6, 16, 144, 256, 3072>;
using D256 = Family<double, 6, 8, 96, 256, 1536>;

}  // namespace

void gemm(bool ta, bool tb, long M, long N, long K, float alpha, const float* A, long lda, const float* B, long ldb,
          float beta, float* C, long ldc) {
  if (has_avx512())
    gemm_impl(F512{&micro_avx512_f}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  else if (has_avx2_fma())
    gemm_impl(F256{&micro_avx2_f}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  else
    gemm_impl(F256{&micro_scalar<float, 6, 16>}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}
void gemm(bool ta, bool tb, long M, long N, long K, double alpha, const double* A, long lda, const double* B, long ldb,
          double beta, double* C, long ldc) {
  if (has_avx512())
    gemm_impl(D512{&micro_avx512_d}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  else if (has_avx2_fma())
    gemm_impl(D256{&micro_avx2_d}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  else
    gemm_impl(D256{&micro_scalar<double, 6, 8>}, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}
bool gemm_uses_avx2() { return has_avx2_fma(); }
bool gemm_uses_avx512() { return has_avx512(); }

}  // namespace cpu
}  // namespace dcnn_native
