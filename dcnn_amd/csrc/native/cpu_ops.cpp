// Native CPU compute backend: elementwise / reduction / layout ops and the layer kernels
// (convolution, dense, batch & group norm, pooling, activations, losses, optimizers), templated
// on float and double, NCHW contiguous, run on the native ThreadPool.
//
// Reference (what, not how): src/ops/cpu/skernels.cpp:22-1493 + dkernels.cpp (AVX2 fp32/fp64
// elementwise & reductions), include/tensor/cpu/tensor_ops.hpp:283 (im2col / col2im / pad / crop),
// src/nn/layers_impl/cpu/conv2d_ops.cpp:19-67 (im2col + SGEMM conv), batchnorm_ops.cpp,
// maxpool_ops.cpp, avgpool_ops.cpp, src/nn/loss_impl/cpu/loss_ops.cpp, include/nn/optimizers.hpp.
//
// Design: convolution works one sample at a time (per-sample im2col panel, reused from a
// thread-local buffer, then the blocked GEMM of cpu_gemm.cpp writes straight into the NCHW output
// — no CNHW round trip); samples are spread over the pool when there are enough of them, else
// each sample's GEMM is parallel. Every reduction (weight gradients, BN/GN statistics, losses,
// generic sums) uses fixed chunk boundaries and combines the chunk partials in chunk order, so
// results are bit-identical for any thread count.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "cpu_kernels.h"
#include "threadpool.h"

namespace dcnn_native {
namespace cpu {

namespace {

constexpr long kGrain = 16384;  // elements per chunk for streaming loops

template <typename F>
void for_chunks(long n, long grain, F&& fn) {
  parallel_for(0, n, grain, [&](long lo, long hi) { fn(lo, hi); });
}

// Deterministic sum of f(i) over [0, n): fixed chunking, chunk partials in double, summed in order.
template <typename F>
double det_sum(long n, F&& f) {
  const long nch = reduction_chunks(n, kGrain);
  if (nch <= 0) return 0.0;
  std::vector<double> part(nch, 0.0);
  ThreadPool::instance().run(nch, [&](long k) {
    const long lo = k * n / nch, hi = (k + 1) * n / nch;
    double s = 0.0;
    for (long i = lo; i < hi; ++i) s += f(i);
    part[k] = s;
  });
  double s = 0.0;
  for (double v : part) s += v;
  return s;
}

inline int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

}  // namespace

// ------------------------------------------------------------------ elementwise
// codes shared with the GPU generic ops (ops/generic.py, csrc/kernels/ops.hip). The op switch is
// resolved once per call; each op body is a plain loop the compiler vectorises.
namespace {
template <typename T, typename F>
void map1(const T* a, T* c, long n, F f) {
  for_chunks(n, kGrain, [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) c[i] = f(a[i]);
  });
}
template <typename T, typename F>
void map2(const T* a, const T* b, T* c, long n, F f) {
  for_chunks(n, kGrain, [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) c[i] = f(a[i], b[i]);
  });
}
}  // namespace

template <typename T>
void elementwise(int mode, int op, const T* a, const T* b, T* c, long n, double s0, double s1) {
  const T x0 = (T)s0, x1 = (T)s1;
  if (mode == 0 || mode == 1) {
    auto bin = [&](auto f) {
      if (mode == 0)
        map2(a, b, c, n, f);
      else
        map1(a, c, n, [&](T u) { return f(u, x0); });
    };
    switch (op) {
      case 0: return bin([](T u, T v) { return u + v; });
      case 1: return bin([](T u, T v) { return u - v; });
      case 2: return bin([](T u, T v) { return u * v; });
      case 3: return bin([](T u, T v) { return u / v; });
      case 4: return bin([](T u, T v) { return u < v ? u : v; });
      case 5: return bin([](T u, T v) { return u > v ? u : v; });
      case 6: return bin([](T u, T v) { return (T)(u == v); });
      case 7: return bin([](T u, T v) { return (T)(u > v); });
    }
    throw std::invalid_argument("elementwise: bad binary op");
  }
  if (mode == 2) {
    switch (op) {
      case 16: return map1(a, c, n, [](T u) { return std::sqrt(u); });
      case 17: return map1(a, c, n, [](T u) { return T(1) / std::sqrt(u); });
      case 18: return map1(a, c, n, [](T u) { return T(1) / u; });
      case 19: return map1(a, c, n, [](T u) { return std::abs(u); });
      case 20: return map1(a, c, n, [](T u) { return -u; });
      case 21: return map1(a, c, n, [](T u) { return std::exp(u); });
      case 22: return map1(a, c, n, [](T u) { return std::log(u); });
      case 23: return map1(a, c, n, [](T u) { return u; });
      case 48: return map1(a, c, n, [&](T u) { return u < x0 ? x0 : (u > x1 ? x1 : u); });  // clamp
      case 49: return map1(a, c, n, [&](T u) { return (u - x0) * x1; });                   // sub_mul
      case 50: return map1(a, c, n, [&](T u) { return u * x0 + x1; });                     // mul_add
    }
    throw std::invalid_argument("elementwise: bad unary op");
  }
  if (mode == 3) {  // ternary, in place on c
    for_chunks(n, kGrain, [&](long lo, long hi) {
      if (op == 32)
        for (long i = lo; i < hi; ++i) c[i] = a[i] * b[i] + c[i];
      else if (op == 33)
        for (long i = lo; i < hi; ++i) c[i] = a[i] * b[i] - c[i];
      else
        for (long i = lo; i < hi; ++i) c[i] = c[i] - a[i] * b[i];
    });
    return;
  }
  if (mode == 4) {  // axpy: c += s0 * a
    for_chunks(n, kGrain, [&](long lo, long hi) {
      for (long i = lo; i < hi; ++i) c[i] += x0 * a[i];
    });
    return;
  }
  throw std::invalid_argument("elementwise: bad mode");
}

// op 0 sum(a), 1 dot(a, b), 2 sum(a^2), 3 sum((a-b)^2)
template <typename T>
double reduce(int op, const T* a, const T* b, long n) {
  switch (op) {
    case 0: return det_sum(n, [&](long i) { return (double)a[i]; });
    case 1: return det_sum(n, [&](long i) { return (double)a[i] * b[i]; });
    case 2: return det_sum(n, [&](long i) { return (double)a[i] * a[i]; });
    case 3: return det_sum(n, [&](long i) { const double d = (double)a[i] - b[i]; return d * d; });
  }
  throw std::invalid_argument("reduce: bad op");
}

// Philox-4x32-10, bit-identical to the GPU fill (csrc/kernels/common.h Philox): the same seed
// gives the same numbers on either device.
static inline void philox(uint64_t seed, uint64_t ctr, uint32_t out[4]) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x6a09e667u, c3 = 0xbb67ae85u;
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
static inline float u01(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

template <typename T>
void fill_random(T* out, long n, uint64_t seed, double a, double b, int normal) {
  const long nq = (n + 3) / 4;
  for_chunks(nq, 4096, [&](long lo, long hi) {
    for (long q = lo; q < hi; ++q) {
      uint32_t r[4];
      philox(seed, (uint64_t)q, r);
      float v[4];
      if (normal) {
        const float uu1 = std::max(u01(r[0]), 1e-12f), uu2 = u01(r[1]);
        const float uu3 = std::max(u01(r[2]), 1e-12f), uu4 = u01(r[3]);
        const float r1 = std::sqrt(-2.f * std::log(uu1)), r2 = std::sqrt(-2.f * std::log(uu3));
        v[0] = r1 * std::cos(6.28318530718f * uu2);
        v[1] = r1 * std::sin(6.28318530718f * uu2);
        v[2] = r2 * std::cos(6.28318530718f * uu4);
        v[3] = r2 * std::sin(6.28318530718f * uu4);
        for (int k = 0; k < 4; ++k) v[k] = (float)a + (float)b * v[k];
      } else {
        for (int k = 0; k < 4; ++k) v[k] = (float)a + ((float)b - (float)a) * u01(r[k]);
      }
      for (int k = 0; k < 4; ++k)
        if (q * 4 + k < n) out[q * 4 + k] = (T)v[k];
    }
  });
}

// ------------------------------------------------------------------ layout
template <typename T>
void transpose2d(const T* in, T* out, long batch, long rows, long cols) {
  constexpr long B = 32;
  const long tr = (rows + B - 1) / B, tc = (cols + B - 1) / B;
  parallel_for(0, batch * tr * tc, 1, [&](long lo, long hi) {
    for (long t = lo; t < hi; ++t) {
      const long z = t / (tr * tc), r0 = (t / tc % tr) * B, c0 = (t % tc) * B;
      const T* src = in + z * rows * cols;
      T* dst = out + z * rows * cols;
      for (long r = r0; r < std::min(rows, r0 + B); ++r)
        for (long c = c0; c < std::min(cols, c0 + B); ++c) dst[c * rows + r] = src[r * cols + c];
    }
  });
}

// [A][B][HW] -> [B][A][HW]  (NCHW <-> CNHW)
template <typename T>
void swap01(const T* in, T* out, long A, long Bn, long HW) {
  parallel_for(0, A * Bn, 1, [&](long lo, long hi) {
    for (long t = lo; t < hi; ++t) {
      const long a = t / Bn, b = t % Bn;
      std::memcpy(out + (b * A + a) * HW, in + (a * Bn + b) * HW, HW * sizeof(T));
    }
  });
}

template <typename T>
void pad2d(const T* x, T* y, long NC, int H, int W, int ph, int pw, double value) {
  const int OH = H + 2 * ph, OW = W + 2 * pw;
  parallel_for(0, NC, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      T* o = y + p * OH * OW;
      const T* s = x + p * H * W;
      std::fill(o, o + (long)OH * OW, (T)value);
      for (int h = 0; h < H; ++h) std::memcpy(o + (long)(h + ph) * OW + pw, s + (long)h * W, W * sizeof(T));
    }
  });
}

template <typename T>
void crop2d(const T* x, T* y, long NC, int H, int W, int top, int left, int OH, int OW) {
  parallel_for(0, NC, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p)
      for (int h = 0; h < OH; ++h)
        std::memcpy(y + (p * OH + h) * OW, x + (p * H + h + top) * (long)W + left, OW * sizeof(T));
  });
}

// ------------------------------------------------------------------ im2col / col2im
// One sample: col[(c, kh, kw)][oh * OW + ow]
template <typename T>
static void im2col_one(const T* x, T* col, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW, int OH,
                       int OW) {
  for (int c = 0; c < C; ++c)
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw) {
        T* dst = col + (((long)c * KH + kh) * KW + kw) * OH * OW;
        const T* src = x + (long)c * H * W;
        for (int oh = 0; oh < OH; ++oh) {
          const int iy = oh * SH - PH + kh;
          T* d = dst + (long)oh * OW;
          if (iy < 0 || iy >= H) {
            std::fill(d, d + OW, T(0));
            continue;
          }
          const T* srow = src + (long)iy * W;
          if (SW == 1) {
            const int ox0 = std::max(0, PW - kw), ox1 = std::min(OW, W + PW - kw);
            for (int ow = 0; ow < std::min(ox0, OW); ++ow) d[ow] = T(0);
            if (ox1 > ox0) std::memcpy(d + ox0, srow + ox0 - PW + kw, (ox1 - ox0) * sizeof(T));
            for (int ow = std::max(ox1, 0); ow < OW; ++ow) d[ow] = T(0);
          } else {
            for (int ow = 0; ow < OW; ++ow) {
              const int ix = ow * SW - PW + kw;
              d[ow] = (ix >= 0 && ix < W) ? srow[ix] : T(0);
            }
          }
        }
      }
}

template <typename T>
static void col2im_one(const T* col, T* x, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW, int OH,
                       int OW) {
  std::fill(x, x + (long)C * H * W, T(0));
  for (int c = 0; c < C; ++c)
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw) {
        const T* src = col + (((long)c * KH + kh) * KW + kw) * OH * OW;
        T* dst = x + (long)c * H * W;
        for (int oh = 0; oh < OH; ++oh) {
          const int iy = oh * SH - PH + kh;
          if (iy < 0 || iy >= H) continue;
          T* drow = dst + (long)iy * W;
          const T* s = src + (long)oh * OW;
          for (int ow = 0; ow < OW; ++ow) {
            const int ix = ow * SW - PW + kw;
            if (ix >= 0 && ix < W) drow[ix] += s[ow];
          }
        }
      }
}

// Reference layout (tensor_kernels.cu:18 / tensor_ops.hpp:283): col[(c,kh,kw)][n*OH*OW + oh*OW + ow]
template <typename T>
void im2col(const T* x, T* col, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const long L = (long)OH * OW, rows = (long)C * KH * KW;
  parallel_for(0, N, 1, [&](long lo, long hi) {
    std::vector<T> tmp(rows * L);
    for (long n = lo; n < hi; ++n) {
      im2col_one(x + n * C * H * W, tmp.data(), C, H, W, KH, KW, SH, SW, PH, PW, OH, OW);
      for (long r = 0; r < rows; ++r) std::memcpy(col + r * N * L + n * L, tmp.data() + r * L, L * sizeof(T));
    }
  });
}

template <typename T>
void col2im(const T* col, T* x, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const long L = (long)OH * OW, rows = (long)C * KH * KW;
  parallel_for(0, N, 1, [&](long lo, long hi) {
    std::vector<T> tmp(rows * L);
    for (long n = lo; n < hi; ++n) {
      for (long r = 0; r < rows; ++r) std::memcpy(tmp.data() + r * L, col + r * N * L + n * L, L * sizeof(T));
      col2im_one(tmp.data(), x + n * C * H * W, C, H, W, KH, KW, SH, SW, PH, PW, OH, OW);
    }
  });
}

// ------------------------------------------------------------------ convolution
namespace {
// per-thread reusable buffers (slot 0: per-sample im2col panels; slots 1/2: the batched
// schedule's column matrix and channel-major output): no per-call allocation, zeroing or page
// faults of multi-MB vectors
template <typename T, int SLOT = 0>
std::vector<T>& scratch(size_t n) {
  thread_local std::vector<T> buf;
  if (buf.size() < n) buf.resize(n);
  return buf;
}
bool is_1x1_direct(int KH, int KW, int SH, int SW, int PH, int PW) {
  return KH == 1 && KW == 1 && SH == 1 && SW == 1 && PH == 0 && PW == 0;
}
// Run fn(n) for every sample: across the pool when there are enough samples, otherwise in
// order with each sample's GEMM using the pool itself.
template <typename F>
void per_sample(long N, F&& fn) {
  if (N >= get_num_threads() && !in_parallel_region()) {
    ThreadPool::instance().run(N, [&](long n) { fn(n); });
  } else {
    for (long n = 0; n < N; ++n) fn(n);
  }
}
}  // namespace

// Two schedules:
// * batched (small feature maps, where one sample's GEMM is too small to run efficiently):
//   col[K][N*L] for the whole batch (the reference's layout), ONE GEMM W[Co][K] @ col -> Y'[Co][N*L],
//   then CNHW -> NCHW; the backward runs the weight gradient as one GEMM over the N*L axis;
// * per sample (large feature maps): a per-sample im2col panel from a thread-local buffer and
//   the GEMM writing straight into the NCHW output.
namespace {
template <typename T>
bool conv_batched(long N, long K, long L) {
  return L < 1024 && (double)K * N * L * sizeof(T) <= 256.0 * (1 << 20);
}
template <typename T>
void add_bias_nchw(T* y, const T* bias, long N, long Co, long L) {
  parallel_for(0, N * Co, std::max(1L, 8192 / std::max(1L, L)), [&](long lo, long hi) {
    for (long t = lo; t < hi; ++t) {
      T* r = y + t * L;
      const T bv = bias[t % Co];
      for (long i = 0; i < L; ++i) r[i] += bv;
    }
  });
}
}  // namespace

template <typename T>
void conv2d_fwd(const T* x, const T* w, const T* bias, T* y, int N, int C, int H, int W, int Co, int KH, int KW, int SH,
                int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const long L = (long)OH * OW, K = (long)C * KH * KW;
  const bool direct = is_1x1_direct(KH, KW, SH, SW, PH, PW);
  if (conv_batched<T>(N, K, L) && N > 1) {
    auto& col = scratch<T, 1>((size_t)K * N * L);
    auto& yc = scratch<T, 2>((size_t)Co * N * L);
    im2col(x, col.data(), N, C, H, W, KH, KW, SH, SW, PH, PW);
    gemm(false, false, Co, N * L, K, T(1), w, K, col.data(), N * L, T(0), yc.data(), N * L);
    swap01(yc.data(), y, Co, N, L);
    if (bias) add_bias_nchw(y, bias, N, Co, L);
    return;
  }
  per_sample(N, [&](long n) {
    const T* xn = x + n * C * H * W;
    T* yn = y + n * Co * L;
    const T* col = xn;
    if (!direct) {
      auto& buf = scratch<T>(K * L);
      im2col_one(xn, buf.data(), C, H, W, KH, KW, SH, SW, PH, PW, OH, OW);
      col = buf.data();
    }
    gemm(false, false, Co, L, K, T(1), w, K, col, L, T(0), yn, L);
  });
  if (bias) add_bias_nchw(y, bias, N, Co, L);
}

// dx (overwrite, may be null), dw += sum_n dy_n @ col_n^T, db += sum dy (may be null).
// The weight gradient is reduced over fixed sample chunks in chunk order (deterministic).
template <typename T>
void conv2d_bwd(const T* x, const T* w, const T* dy, T* dx, T* dw, T* db, int N, int C, int H, int W, int Co, int KH,
                int KW, int SH, int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const long L = (long)OH * OW, K = (long)C * KH * KW;
  const bool direct = is_1x1_direct(KH, KW, SH, SW, PH, PW);
  // ---- bias gradient (per channel, samples then pixels in order)
  if (db) {
    parallel_for(0, Co, 1, [&](long lo, long hi) {
      for (long co = lo; co < hi; ++co) {
        double s = 0.0;
        for (long n = 0; n < N; ++n) {
          const T* r = dy + (n * Co + co) * L;
          for (long i = 0; i < L; ++i) s += r[i];
        }
        db[co] += (T)s;
      }
    });
  }
  if (conv_batched<T>(N, K, L) && N > 1) {
    auto& col = scratch<T, 1>((size_t)K * N * L);
    auto& dyc = scratch<T, 2>((size_t)Co * N * L);
    im2col(x, col.data(), N, C, H, W, KH, KW, SH, SW, PH, PW);
    swap01(dy, dyc.data(), N, Co, L);  // [Co][N*L]
    gemm(false, true, Co, K, N * L, T(1), dyc.data(), N * L, col.data(), N * L, T(1), dw, K);
    if (dx) {
      gemm(true, false, K, N * L, Co, T(1), w, K, dyc.data(), N * L, T(0), col.data(), N * L);
      col2im(col.data(), dx, N, C, H, W, KH, KW, SH, SW, PH, PW);
    }
    return;
  }
  // ---- weight gradient: fixed sample chunks (independent of the thread count), each chunk's
  // partial in its own slab, slabs summed in chunk order
  const long nch = std::min<long>(N, 16);
  const bool spread = nch > 1;
  std::vector<T> part(spread ? (size_t)nch * Co * K : 0);
  auto wgrad_range = [&](long lo, long hi, T* acc, T beta0) {
    T beta = beta0;
    for (long n = lo; n < hi; ++n) {
      const T* col = x + n * C * H * W;
      if (!direct) {
        auto& buf = scratch<T>(K * L);
        im2col_one(x + n * C * H * W, buf.data(), C, H, W, KH, KW, SH, SW, PH, PW, OH, OW);
        col = buf.data();
      }
      gemm(false, true, Co, K, L, T(1), dy + n * Co * L, L, col, L, beta, acc, K);
      beta = T(1);
    }
  };
  if (spread) {
    ThreadPool::instance().run(nch, [&](long k) {
      wgrad_range(k * N / nch, (k + 1) * N / nch, part.data() + k * Co * K, T(0));
    });
    const long WN = (long)Co * K;
    for_chunks(WN, kGrain, [&](long lo, long hi) {
      for (long k = 0; k < nch; ++k) {
        const T* p = part.data() + k * WN;
        for (long i = lo; i < hi; ++i) dw[i] += p[i];
      }
    });
  } else {
    wgrad_range(0, N, dw, T(1));
  }
  // ---- data gradient: col_n = W^T @ dy_n, scattered back
  if (dx) {
    per_sample(N, [&](long n) {
      T* dxn = dx + n * C * H * W;
      if (direct) {
        gemm(true, false, C, L, Co, T(1), w, K, dy + n * Co * L, L, T(0), dxn, L);
        return;
      }
      auto& buf = scratch<T>(K * L);
      gemm(true, false, K, L, Co, T(1), w, K, dy + n * Co * L, L, T(0), buf.data(), L);
      col2im_one(buf.data(), dxn, C, H, W, KH, KW, SH, SW, PH, PW, OH, OW);
    });
  }
}

// ------------------------------------------------------------------ dense
template <typename T>
void dense_fwd(const T* x, const T* w, const T* bias, T* y, long N, long In, long Out) {
  gemm(false, true, N, Out, In, T(1), x, In, w, In, T(0), y, Out);
  if (bias)
    for_chunks(N, std::max(1L, kGrain / std::max(1L, Out)), [&](long lo, long hi) {
      for (long i = lo; i < hi; ++i)
        for (long o = 0; o < Out; ++o) y[i * Out + o] += bias[o];
    });
}

template <typename T>
void dense_bwd(const T* x, const T* w, const T* dy, T* dx, T* dw, T* db, long N, long In, long Out) {
  gemm(true, false, Out, In, N, T(1), dy, Out, x, In, T(1), dw, In);
  if (db)
    parallel_for(0, Out, 64, [&](long lo, long hi) {
      for (long o = lo; o < hi; ++o) {
        double s = 0.0;
        for (long i = 0; i < N; ++i) s += dy[i * Out + o];
        db[o] += (T)s;
      }
    });
  if (dx) gemm(false, false, N, In, Out, T(1), dy, Out, w, In, T(0), dx, In);
}

// ------------------------------------------------------------------ batch norm
// Per channel: two-pass statistics in double (mean, then centred second moment), fixed order.
template <typename T>
void batchnorm_fwd(const T* x, T* y, long N, long C, long HW, const T* gamma, const T* beta, double eps, int training,
                   T* running_mean, T* running_var, double momentum, T* save_mean, T* save_istd, int relu,
                   const T* residual) {
  parallel_for(0, C, 1, [&](long lo, long hi) {
    for (long c = lo; c < hi; ++c) {
      double mean, var;
      if (training) {
        double s = 0.0;
        for (long n = 0; n < N; ++n) {
          const T* r = x + (n * C + c) * HW;
          for (long i = 0; i < HW; ++i) s += r[i];
        }
        const double M = (double)N * HW;
        mean = s / M;
        double q = 0.0;
        for (long n = 0; n < N; ++n) {
          const T* r = x + (n * C + c) * HW;
          for (long i = 0; i < HW; ++i) {
            const double d = r[i] - mean;
            q += d * d;
          }
        }
        var = q / M;
        if (running_mean) {
          const double unb = var * M / std::max(M - 1.0, 1.0);
          running_mean[c] = (T)((1.0 - momentum) * running_mean[c] + momentum * mean);
          running_var[c] = (T)((1.0 - momentum) * running_var[c] + momentum * unb);
        }
      } else {
        mean = running_mean[c];
        var = running_var[c];
      }
      const double istd = 1.0 / std::sqrt(var + eps);
      if (save_mean) save_mean[c] = (T)mean;
      if (save_istd) save_istd[c] = (T)istd;
      const T sc = (T)(istd * (gamma ? (double)gamma[c] : 1.0));
      const T sh = (T)((beta ? (double)beta[c] : 0.0) - mean * istd * (gamma ? (double)gamma[c] : 1.0));
      for (long n = 0; n < N; ++n) {
        const long off = (n * C + c) * HW;
        const T* r = x + off;
        T* o = y + off;
        const T* res = residual ? residual + off : nullptr;
        for (long i = 0; i < HW; ++i) {
          T v = r[i] * sc + sh;
          if (res) v += res[i];
          o[i] = relu && v < T(0) ? T(0) : v;
        }
      }
    }
  });
}

// dy masked by (yout > 0) when yout is given (fused ReLU); masked_out receives that masked dy.
template <typename T>
void batchnorm_bwd(const T* x, const T* dy, const T* yout, const T* mean, const T* istd, const T* gamma, T* dx,
                   T* dgamma, T* dbeta, T* masked_out, long N, long C, long HW, int training) {
  parallel_for(0, C, 1, [&](long lo, long hi) {
    for (long c = lo; c < hi; ++c) {
      const double mu = mean[c], is = istd[c];
      double sdy = 0.0, sdyx = 0.0;
      for (long n = 0; n < N; ++n) {
        const long off = (n * C + c) * HW;
        for (long i = 0; i < HW; ++i) {
          T d = dy[off + i];
          if (yout && !(yout[off + i] > T(0))) d = T(0);
          if (masked_out) masked_out[off + i] = d;
          sdy += d;
          sdyx += (double)d * ((x[off + i] - mu) * is);
        }
      }
      if (dgamma) dgamma[c] += (T)sdyx;
      if (dbeta) dbeta[c] += (T)sdy;
      if (!dx) continue;
      const double g = gamma ? (double)gamma[c] : 1.0;
      const double M = (double)N * HW;
      const double a = g * is, m1 = sdy / M, m2 = sdyx / M;
      for (long n = 0; n < N; ++n) {
        const long off = (n * C + c) * HW;
        for (long i = 0; i < HW; ++i) {
          T d = dy[off + i];
          if (yout && !(yout[off + i] > T(0))) d = T(0);
          if (training) {
            const double xh = (x[off + i] - mu) * is;
            dx[off + i] = (T)(a * (d - m1 - xh * m2));
          } else {
            dx[off + i] = (T)(a * d);
          }
        }
      }
    }
  });
}

// ------------------------------------------------------------------ group norm
template <typename T>
void groupnorm_fwd(const T* x, T* y, long N, long C, long HW, long G, const T* gamma, const T* beta, double eps,
                   T* save_mean, T* save_istd) {
  const long cg = C / G, len = cg * HW;
  parallel_for(0, N * G, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      const long n = p / G, g = p % G;
      const T* r = x + (n * C + g * cg) * HW;
      double s = 0.0;
      for (long i = 0; i < len; ++i) s += r[i];
      const double mean = s / len;
      double q = 0.0;
      for (long i = 0; i < len; ++i) {
        const double d = r[i] - mean;
        q += d * d;
      }
      const double istd = 1.0 / std::sqrt(q / len + eps);
      save_mean[p] = (T)mean;
      save_istd[p] = (T)istd;
      T* o = y + (n * C + g * cg) * HW;
      for (long cc = 0; cc < cg; ++cc) {
        const long c = g * cg + cc;
        const double ga = gamma ? (double)gamma[c] : 1.0, be = beta ? (double)beta[c] : 0.0;
        const T sc = (T)(istd * ga), sh = (T)(be - mean * istd * ga);
        for (long i = 0; i < HW; ++i) o[cc * HW + i] = r[cc * HW + i] * sc + sh;
      }
    }
  });
}

template <typename T>
void groupnorm_bwd(const T* x, const T* dy, const T* mean, const T* istd, const T* gamma, T* dx, T* dgamma, T* dbeta,
                   long N, long C, long HW, long G) {
  const long cg = C / G, len = cg * HW;
  if (dgamma || dbeta)
    parallel_for(0, C, 1, [&](long lo, long hi) {
      for (long c = lo; c < hi; ++c) {
        const long g = c / cg;
        double sg = 0.0, sb = 0.0;
        for (long n = 0; n < N; ++n) {
          const double mu = mean[n * G + g], is = istd[n * G + g];
          const T* d = dy + (n * C + c) * HW;
          const T* xr = x + (n * C + c) * HW;
          for (long i = 0; i < HW; ++i) {
            sb += d[i];
            sg += (double)d[i] * ((xr[i] - mu) * is);
          }
        }
        if (dgamma) dgamma[c] += (T)sg;
        if (dbeta) dbeta[c] += (T)sb;
      }
    });
  parallel_for(0, N * G, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      const long n = p / G, g = p % G;
      const double mu = mean[p], is = istd[p];
      const long base = (n * C + g * cg) * HW;
      double m1 = 0.0, m2 = 0.0;
      for (long cc = 0; cc < cg; ++cc) {
        const double ga = gamma ? (double)gamma[g * cg + cc] : 1.0;
        for (long i = 0; i < HW; ++i) {
          const double d = dy[base + cc * HW + i] * ga;
          m1 += d;
          m2 += d * ((x[base + cc * HW + i] - mu) * is);
        }
      }
      m1 /= len;
      m2 /= len;
      for (long cc = 0; cc < cg; ++cc) {
        const double ga = gamma ? (double)gamma[g * cg + cc] : 1.0;
        for (long i = 0; i < HW; ++i) {
          const long k = base + cc * HW + i;
          const double xh = (x[k] - mu) * is;
          dx[k] = (T)(is * (dy[k] * ga - m1 - xh * m2));
        }
      }
    }
  });
}

// ------------------------------------------------------------------ pooling
// argmax index = iy * W + ix within the plane (first maximum in window order), -1 for an
// all-padding window
template <typename T>
void maxpool_fwd(const T* x, T* y, int32_t* idx, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH,
                 int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  parallel_for(0, NC, std::max(1L, 4096L / std::max(1, H * W)), [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      const T* xp = x + p * H * W;
      T* yp = y + p * OH * OW;
      int32_t* ip = idx + p * OH * OW;
      for (int oh = 0; oh < OH; ++oh) {
        const int y0 = std::max(0, oh * SH - PH), y1 = std::min(H, oh * SH - PH + KH);
        for (int ow = 0; ow < OW; ++ow) {
          const int x0 = std::max(0, ow * SW - PW), x1 = std::min(W, ow * SW - PW + KW);
          int32_t bi = -1;
          T best = T(0);
          for (int iy = y0; iy < y1; ++iy) {
            const T* r = xp + iy * W;
            for (int ix = x0; ix < x1; ++ix)
              if (bi < 0 || r[ix] > best) {  // ties: first element in window order
                best = r[ix];
                bi = iy * W + ix;
              }
          }
          yp[oh * OW + ow] = best;
          ip[oh * OW + ow] = bi;
        }
      }
    }
  });
}

// per plane, scatter-add in output order (overlapping windows stay deterministic)
template <typename T>
void maxpool_bwd(const T* dy, const int32_t* idx, T* dx, long NC, int H, int W, int OH, int OW) {
  parallel_for(0, NC, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      T* d = dx + p * H * W;
      std::fill(d, d + (long)H * W, T(0));
      const T* g = dy + p * OH * OW;
      const int32_t* ix = idx + p * OH * OW;
      for (long o = 0; o < (long)OH * OW; ++o)
        if (ix[o] >= 0) d[ix[o]] += g[o];
    }
  });
}

// count_include_pad semantics (divisor KH*KW), as the GPU kernel and the reference
template <typename T>
void avgpool_fwd(const T* x, T* y, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const T inv = T(1) / T(KH * KW);
  parallel_for(0, NC, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      const T* xp = x + p * H * W;
      for (int oh = 0; oh < OH; ++oh)
        for (int ow = 0; ow < OW; ++ow) {
          T s = 0;
          for (int kh = 0; kh < KH; ++kh) {
            const int iy = oh * SH - PH + kh;
            if (iy < 0 || iy >= H) continue;
            for (int kw = 0; kw < KW; ++kw) {
              const int ix = ow * SW - PW + kw;
              if (ix >= 0 && ix < W) s += xp[iy * W + ix];
            }
          }
          y[(p * OH + oh) * OW + ow] = s * inv;
        }
    }
  });
}

template <typename T>
void avgpool_bwd(const T* dy, T* dx, long NC, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW) {
  const int OH = out_dim(H, KH, SH, PH), OW = out_dim(W, KW, SW, PW);
  const T inv = T(1) / T(KH * KW);
  parallel_for(0, NC, 1, [&](long lo, long hi) {
    for (long p = lo; p < hi; ++p) {
      T* d = dx + p * H * W;
      std::fill(d, d + (long)H * W, T(0));
      const T* g = dy + p * OH * OW;
      for (int oh = 0; oh < OH; ++oh)
        for (int ow = 0; ow < OW; ++ow) {
          const T v = g[oh * OW + ow] * inv;
          for (int kh = 0; kh < KH; ++kh) {
            const int iy = oh * SH - PH + kh;
            if (iy < 0 || iy >= H) continue;
            for (int kw = 0; kw < KW; ++kw) {
              const int ix = ow * SW - PW + kw;
              if (ix >= 0 && ix < W) d[iy * W + ix] += v;
            }
          }
        }
    }
  });
}

// ------------------------------------------------------------------ activations
// type: 0 linear, 1 relu, 2 leaky_relu(alpha), 3 elu(alpha), 4 sigmoid, 5 tanh
template <typename T>
void act_fwd(int type, const T* x, T* y, long n, double alpha) {
  const T a = (T)alpha;
  switch (type) {
    case 1: return map1(x, y, n, [](T v) { return v > T(0) ? v : T(0); });
    case 2: return map1(x, y, n, [&](T v) { return v > T(0) ? v : v * a; });
    case 3: return map1(x, y, n, [&](T v) { return v > T(0) ? v : a * (std::exp(v) - T(1)); });
    case 4: return map1(x, y, n, [](T v) { return T(1) / (T(1) + std::exp(-v)); });
    case 5: return map1(x, y, n, [](T v) { return std::tanh(v); });
    default: return map1(x, y, n, [](T v) { return v; });
  }
}

template <typename T>
void act_bwd(int type, const T* x, const T* dy, T* dx, long n, double alpha) {
  const T a = (T)alpha;
  switch (type) {
    case 1: return map2(x, dy, dx, n, [](T v, T g) { return v > T(0) ? g : T(0); });
    case 2: return map2(x, dy, dx, n, [&](T v, T g) { return v > T(0) ? g : g * a; });
    case 3: return map2(x, dy, dx, n, [&](T v, T g) { return v > T(0) ? g : g * a * std::exp(v); });
    case 4: return map2(x, dy, dx, n, [](T v, T g) {
      const T s = T(1) / (T(1) + std::exp(-v));
      return g * s * (T(1) - s);
    });
    case 5: return map2(x, dy, dx, n, [](T v, T g) {
      const T t = std::tanh(v);
      return g * (T(1) - t * t);
    });
    default: return map2(x, dy, dx, n, [](T, T g) { return g; });
  }
}

// softmax over the channel dim at every (n, spatial) position: x [N][C][HW]
template <typename T>
void softmax_channels(const T* x, T* y, long N, long C, long HW) {
  parallel_for(0, N * HW, 256, [&](long lo, long hi) {
    for (long t = lo; t < hi; ++t) {
      const long n = t / HW, s = t % HW;
      const T* xp = x + n * C * HW + s;
      T* yp = y + n * C * HW + s;
      T m = xp[0];
      for (long c = 1; c < C; ++c) m = std::max(m, xp[c * HW]);
      double z = 0.0;
      for (long c = 0; c < C; ++c) z += std::exp((double)xp[c * HW] - m);
      for (long c = 0; c < C; ++c) yp[c * HW] = (T)(std::exp((double)xp[c * HW] - m) / z);
    }
  });
}

template <typename T>
void softmax_channels_bwd(const T* y, const T* dy, T* dx, long N, long C, long HW) {
  parallel_for(0, N * HW, 256, [&](long lo, long hi) {
    for (long t = lo; t < hi; ++t) {
      const long n = t / HW, s = t % HW;
      const long base = n * C * HW + s;
      double dot = 0.0;
      for (long c = 0; c < C; ++c) dot += (double)y[base + c * HW] * dy[base + c * HW];
      for (long c = 0; c < C; ++c) dx[base + c * HW] = (T)(y[base + c * HW] * (dy[base + c * HW] - dot));
    }
  });
}

// ------------------------------------------------------------------ losses
// kind: 0 crossentropy (probabilities, eps clamp), 1 softmax_crossentropy, 2 mse, 3 mae, 4 huber(delta)
// targets either one-hot rows (target != null) or integer labels. Returns the mean loss; writes
// grad (may be null) and the correct count (argmax match).
template <typename T>
double loss_fused(int kind, const T* pred, const T* target, const int64_t* labels, T* grad, long N, long C,
                  double param, long* correct) {
  std::vector<double> lrow(N, 0.0);
  std::vector<int> hit(N, 0);
  const bool regression = kind >= 2;
  const double gscale = regression ? 1.0 / ((double)N * C) : 1.0 / N;
  parallel_for(0, N, 16, [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) {
      const T* p = pred + i * C;
      auto tgt = [&](long c) -> double {
        return target ? (double)target[i * C + c] : (double)(labels[i] == c);
      };
      long hot = -1;
      for (long c = 0; c < C; ++c)
        if (tgt(c) > 0.5) {
          hot = c;
          break;
        }
      long am = 0;
      for (long c = 1; c < C; ++c)
        if (p[c] > p[am]) am = c;
      long tam = 0;
      for (long c = 1; c < C; ++c)
        if (tgt(c) > tgt(tam)) tam = c;
      hit[i] = am == tam;
      double l = 0.0;
      if (kind == 1) {
        double m = p[0];
        for (long c = 1; c < C; ++c) m = std::max(m, (double)p[c]);
        double z = 0.0;
        for (long c = 0; c < C; ++c) z += std::exp((double)p[c] - m);
        const double lse = m + std::log(z);
        if (hot >= 0) l = lse - p[hot];
        if (grad)
          for (long c = 0; c < C; ++c) grad[i * C + c] = (T)((std::exp((double)p[c] - lse) - tgt(c)) * gscale);
      } else if (kind == 0) {
        if (hot >= 0) l = -std::log(std::min(std::max((double)p[hot], param), 1.0 - param));
        if (grad)
          for (long c = 0; c < C; ++c) grad[i * C + c] = (T)((p[c] - tgt(c)) * gscale);
      } else {
        for (long c = 0; c < C; ++c) {
          const double d = (double)p[c] - tgt(c);
          double g;
          if (kind == 2) {
            l += d * d;
            g = 2.0 * d;
          } else if (kind == 3) {
            l += std::abs(d);
            g = d > 0 ? 1.0 : -1.0;
          } else {
            const double ad = std::abs(d);
            l += ad <= param ? 0.5 * d * d : param * ad - 0.5 * param * param;
            g = ad <= param ? d : (d > 0 ? param : -param);
          }
          if (grad) grad[i * C + c] = (T)(g * gscale);
        }
      }
      lrow[i] = l;
    }
  });
  double tot = 0.0;
  long cor = 0;
  for (long i = 0; i < N; ++i) {
    tot += lrow[i];
    cor += hit[i];
  }
  if (correct) *correct = cor;
  return regression ? tot / ((double)N * C) : tot / N;
}

// ------------------------------------------------------------------ optimizers (flat buffers)
template <typename T>
void sgd_step(T* p, const T* g, T* vel, long n, double lr, double momentum) {
  for_chunks(n, kGrain, [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) {
      if (vel) {
        vel[i] = (T)(momentum * vel[i] - lr * g[i]);
        p[i] += vel[i];
      } else {
        p[i] -= (T)(lr * g[i]);
      }
    }
  });
}

template <typename T>
void adam_step(T* p, const T* g, T* m, T* v, long n, double lr, double b1, double b2, double eps, double bc1,
               double bc2, double wd, int decoupled) {
  for_chunks(n, kGrain, [&](long lo, long hi) {
    for (long i = lo; i < hi; ++i) {
      const double gi = g[i];
      m[i] = (T)(b1 * m[i] + (1.0 - b1) * gi);
      v[i] = (T)(b2 * v[i] + (1.0 - b2) * gi * gi);
      double upd = lr * (m[i] / bc1) / (std::sqrt(v[i] / bc2) + eps);
      if (wd > 0) {
        if (decoupled)
          p[i] -= (T)(wd * lr * p[i]);
        else
          upd += wd * lr * p[i];
      }
      p[i] -= (T)upd;
    }
  });
}

// ------------------------------------------------------------------ instantiations
#define DCNN_CPU_INST(T)                                                                                             \
  template void elementwise<T>(int, int, const T*, const T*, T*, long, double, double);                             \
  template double reduce<T>(int, const T*, const T*, long);                                                         \
  template void fill_random<T>(T*, long, uint64_t, double, double, int);                                            \
  template void transpose2d<T>(const T*, T*, long, long, long);                                                     \
  template void swap01<T>(const T*, T*, long, long, long);                                                          \
  template void pad2d<T>(const T*, T*, long, int, int, int, int, double);                                           \
  template void crop2d<T>(const T*, T*, long, int, int, int, int, int, int);                                        \
  template void im2col<T>(const T*, T*, int, int, int, int, int, int, int, int, int, int);                          \
  template void col2im<T>(const T*, T*, int, int, int, int, int, int, int, int, int, int);                          \
  template void conv2d_fwd<T>(const T*, const T*, const T*, T*, int, int, int, int, int, int, int, int, int, int,   \
                              int);                                                                                 \
  template void conv2d_bwd<T>(const T*, const T*, const T*, T*, T*, T*, int, int, int, int, int, int, int, int, int, \
                              int, int);                                                                            \
  template void dense_fwd<T>(const T*, const T*, const T*, T*, long, long, long);                                   \
  template void dense_bwd<T>(const T*, const T*, const T*, T*, T*, T*, long, long, long);                           \
  template void batchnorm_fwd<T>(const T*, T*, long, long, long, const T*, const T*, double, int, T*, T*, double,    \
                                 T*, T*, int, const T*);                                                            \
  template void batchnorm_bwd<T>(const T*, const T*, const T*, const T*, const T*, const T*, T*, T*, T*, T*, long,   \
                                 long, long, int);                                                                  \
  template void groupnorm_fwd<T>(const T*, T*, long, long, long, long, const T*, const T*, double, T*, T*);          \
  template void groupnorm_bwd<T>(const T*, const T*, const T*, const T*, const T*, T*, T*, T*, long, long, long,     \
                                 long);                                                                             \
  template void maxpool_fwd<T>(const T*, T*, int32_t*, long, int, int, int, int, int, int, int, int);               \
  template void maxpool_bwd<T>(const T*, const int32_t*, T*, long, int, int, int, int);                             \
  template void avgpool_fwd<T>(const T*, T*, long, int, int, int, int, int, int, int, int);                         \
  template void avgpool_bwd<T>(const T*, T*, long, int, int, int, int, int, int, int, int);                         \
  template void act_fwd<T>(int, const T*, T*, long, double);                                                        \
  template void act_bwd<T>(int, const T*, const T*, T*, long, double);                                              \
  template void softmax_channels<T>(const T*, T*, long, long, long);                                                \
  template void softmax_channels_bwd<T>(const T*, const T*, T*, long, long, long);                                  \
  template double loss_fused<T>(int, const T*, const T*, const int64_t*, T*, long, long, double, long*);            \
  template void sgd_step<T>(T*, const T*, T*, long, double, double);                                                \
  template void adam_step<T>(T*, const T*, T*, T*, long, double, double, double, double, double, double, double, int);

DCNN_CPU_INST(float)
DCNN_CPU_INST(double)
#undef DCNN_CPU_INST

}  // namespace cpu
}  // namespace dcnn_native
