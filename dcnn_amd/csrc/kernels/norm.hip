// BatchNorm / GroupNorm on NHWC activations (bf16 or fp32 I/O, fp32 statistics).
//
// Reference: src/nn/layers_impl/cuda/batchnorm_ops.cu:17-375 (K20-K24) launches ONE block per
// channel for the statistics (64 blocks on 256 CUs) and stores x_hat. Here:
//   * statistics are split reductions: partial (sum, sumsq) per row-chunk into a slab (or
//     produced for free by the preceding conv's epilogue), then a channel-parallel reduce;
//   * apply = one vectorised pass computing scale/shift per channel in LDS, optionally fusing
//     the residual add and ReLU of a ResNet block; x_hat is never stored (recomputed from x);
//   * backward fuses the ReLU mask into the reduction and the apply, and ACCUMULATES
//     dgamma/dbeta (intended semantics; reference defect G4 overwrote on GPU).
// Semantics kept: biased variance for normalisation, unbiased for the running variance,
// running = (1-m)*running + m*batch (batchnorm_ops.cu:141-153).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "api.h"

namespace dcnn {

template <typename T, int V>
struct VecIO;
template <>
struct VecIO<bf16, 8> {
  __device__ static __forceinline__ void load(const bf16* p, float* f) {
    unpack8(*reinterpret_cast<const uint4*>(p), f);
  }
  __device__ static __forceinline__ void store(bf16* p, const float* f) {
    *reinterpret_cast<uint4*>(p) = pack8(f);
  }
};
template <>
struct VecIO<float, 8> {
  __device__ static __forceinline__ void load(const float* p, float* f) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  __device__ static __forceinline__ void store(float* p, const float* f) {
    reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
};
template <typename T>
struct VecIO1 {
  __device__ static __forceinline__ void load(const T* p, float* f) { f[0] = to_f(p[0]); }
  __device__ static __forceinline__ void store(T* p, const float* f) { p[0] = from_f<T>(f[0]); }
};

template <typename T, int V>
__device__ __forceinline__ void vload(const T* p, float* f) {
  if constexpr (V == 8) VecIO<T, 8>::load(p, f); else VecIO1<T>::load(p, f);
}
template <typename T, int V>
__device__ __forceinline__ void vstore(T* p, const float* f) {
  if constexpr (V == 8) VecIO<T, 8>::store(p, f); else VecIO1<T>::store(p, f);
}

// ---------------------------------------------------------------------------------------
// partial statistics over rows [block*rpb, (block+1)*rpb)
// mode 0: slab[block][3][C] = (count, mean, M2) of x — sums taken about a per-block pivot (the
//         block's first row), merged later with Chan's update: no E[x^2] - mean^2 cancellation
// mode 1 (backward): slab[block][2][C] = (sum dy', sum dy' * xhat) with dy' = dy * (yout > 0 if
//         yout), optionally storing dy' (needed by a residual branch)
// All cross-thread sums run in a fixed order: the result is bit-reproducible.
// ---------------------------------------------------------------------------------------
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_partial_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const T* __restrict__ yout, T* __restrict__ dy_out,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ istd, long R, int C,
                                                         int rpb, float* __restrict__ slab, int mode,
                                                         float* __restrict__ zero_sums) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  if (zero_sums && blockIdx.x == 0)
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) zero_sums[i] = 0.f;
  const int groups = C / V;                       // channel vectors
  const int tpr = groups < 256 ? groups : 256;    // threads per row
  const int rows_conc = 256 / tpr;                // rows processed concurrently
  const int g0 = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  const long r0 = (long)blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  for (int gbase = 0; gbase < groups; gbase += tpr) {
    const int g = gbase + g0;
    float s[V], q[V], pv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) s[v] = q[v] = pv[v] = 0.f;
    float mu[V], is[V];
    if (mode == 1 && g < groups && rsub < rows_conc) {
#pragma unroll
      for (int v = 0; v < V; ++v) { mu[v] = mean[g * V + v]; is[v] = istd[g * V + v]; }
    }
    if (mode == 0 && g < groups && rsub < rows_conc) vload<T, V>(x + r0 * C + (long)g * V, pv);  // pivot row
    if (g < groups && rsub < rows_conc) {
      for (long r = r0 + rsub; r < r1; r += rows_conc) {
        const long o = r * C + (long)g * V;
        float xv[V];
        vload<T, V>(x + o, xv);
        if (mode == 0) {
#pragma unroll
          for (int v = 0; v < V; ++v) { const float d = xv[v] - pv[v]; s[v] += d; q[v] += d * d; }
        } else {
          float d[V];
          vload<T, V>(dy + o, d);
          if (yout) {
            float yo[V];
            vload<T, V>(yout + o, yo);
#pragma unroll
            for (int v = 0; v < V; ++v) d[v] = yo[v] > 0.f ? d[v] : 0.f;
            if (dy_out) vstore<T, V>(dy_out + o, d);
          }
#pragma unroll
          for (int v = 0; v < V; ++v) {
            s[v] += d[v];
            q[v] += d[v] * (xv[v] - mu[v]) * is[v];
          }
        }
      }
    }
    // reduce over rsub through LDS in a fixed order: sh[rows_conc][2][tpr*V] (+ pivots)
    __syncthreads();
    const int width = tpr * V;
    if (g < groups && rsub < rows_conc) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        sh[(rsub * 2 + 0) * width + g0 * V + v] = s[v];
        sh[(rsub * 2 + 1) * width + g0 * V + v] = q[v];
        if (rsub == 0) sh[rows_conc * 2 * width + g0 * V + v] = pv[v];
      }
    }
    __syncthreads();
    const float cnt = (float)(r1 - r0);
    for (int c = threadIdx.x; c < width; c += 256) {
      const int ch = gbase * V + c;
      if (ch < C) {
        float a = 0.f, b = 0.f;
        for (int k = 0; k < rows_conc; ++k) { a += sh[(k * 2 + 0) * width + c]; b += sh[(k * 2 + 1) * width + c]; }
        if (mode == 0) {
          store_welford(slab, blockIdx.x, C, ch, welford_from_shifted(cnt, sh[rows_conc * 2 * width + c], a, b));
        } else {
          slab[((long)blockIdx.x * 2 + 0) * C + ch] = a;
          slab[((long)blockIdx.x * 2 + 1) * C + ch] = b;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Deterministic statistics reduce: slab rows -> stats[2][C]
//   MODE 0: rows are (count, mean, M2) triples -> stats = (mean, biased variance)
//   MODE 1: rows are (sum a, sum b) pairs      -> stats = (sum a, sum b)
// Grid (C/64, ny): lane = channel, each 1024-thread block merges 256 rows (each of its 16 waves
// 16 rows, all loads in flight, pairwise trees in registers and then across the waves in LDS).
// With ny > 1 every block writes its partial and the consumer merges the ny partials (read_stats):
// an in-kernel second level (ticket + agent release/acquire + a serial last block) cost ~10 us per
// reduce on the 32x32 layers. Every merge order is fixed: the result does not depend on timing.
// ---------------------------------------------------------------------------------------
template <int MODE>
struct StatAcc {
  float a, b, c;  // MODE 0: (n, mean, M2); MODE 1: (sum a, sum b, -)
  __device__ __forceinline__ static StatAcc zero() { return StatAcc{0.f, 0.f, 0.f}; }
  __device__ __forceinline__ StatAcc merge(const StatAcc& o) const {
    if constexpr (MODE == 0) {
      const Welford w = welford_merge(Welford{a, b, c}, Welford{o.a, o.b, o.c});
      return StatAcc{w.n, w.mean, w.m2};
    } else {
      return StatAcc{a + o.a, b + o.b, 0.f};
    }
  }
};
constexpr int kStatRW = 16;
// waves per reduce block (rows per block = 16 x waves): fewer rows per block = more blocks in the
// (latency-bound) reduce and more partials for the consumers to merge (8: 0.1-0.6% faster end
// to end than 16 at batch 64 and 256)
// (round 6, tools/gpu/statwaves.sh, same box, 3 alternating reps, ResNet-18 b256 / ResNet-50 b32
// img/s: 8 waves 91.76k-91.98k / 8145-8150, 4 waves 90.92k-91.10k / 8084-8091, 16 waves
// 91.78k-91.98k / 8130-8131)
static const int g_stat_waves = [] {  // (DCNN_STAT_WAVES=4|8|16: experiment override)
  const char* e = std::getenv("DCNN_STAT_WAVES");
  const int v = e ? std::atoi(e) : 8;
  return v == 4 || v == 16 ? v : 8;
}();

// Merge up to kStatRW rows [r0, r1) of channel c: every load in flight at once, then a pairwise
// tree (log2 16 = 4 dependent merge levels instead of a 16-long chain). Fixed order.
template <int MODE, int NR>
__device__ __forceinline__ StatAcc<MODE> stat_tree(const float* __restrict__ src, long stride_row, int r0, int r1,
                                                   int C, int c) {
  constexpr int NV = MODE == 0 ? 3 : 2;
  StatAcc<MODE> v[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const bool ok = r0 + j < r1;
    const float* q = src + (long)(r0 + j) * stride_row + c;
    v[j] = ok ? StatAcc<MODE>{q[0], q[C], NV == 3 ? q[(NV - 1) * C] : 0.f} : StatAcc<MODE>::zero();
  }
#pragma unroll
  for (int w = 1; w < NR; w *= 2)
#pragma unroll
    for (int j = 0; j + w < NR; j += 2 * w) v[j] = v[j].merge(v[j + w]);
  return v[0];
}

// the 16 waves' results in LDS merged by a fixed pairwise tree; result in red[0][lane]
template <int MODE, int WAVES>
__device__ __forceinline__ void stat_tree_lds(StatAcc<MODE> (*red)[64], int w, int lane) {
#pragma unroll
  for (int o = WAVES / 2; o > 0; o >>= 1) {
    __syncthreads();
    if (w < o) red[w][lane] = red[w][lane].merge(red[w + o][lane]);
  }
  __syncthreads();
}

// blockIdx.z selects one of up to two independent reductions of the same C (a residual block's
// tail and projection-shortcut BatchNorms, reduced in one launch); each has its own ny partial
// rows (blocks past a segment's ny exit before any barrier)
template <int MODE, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) bn_stat_reduce_kernel(const float* __restrict__ slab, int rows, int C,
                                                                    float* __restrict__ part,
                                                                    unsigned* __restrict__ ticket,
                                                                    float* __restrict__ out, int ny1,
                                                                    const float* __restrict__ slab2, int rows2,
                                                                    float* __restrict__ part2,
                                                                    float* __restrict__ out2, int ny2) {
  if (blockIdx.z == 1) {
    slab = slab2;
    rows = rows2;
    part = part2;
    out = out2;
    ny1 = ny2;
  }
  if ((int)blockIdx.y >= ny1) return;
  constexpr int NV = MODE == 0 ? 3 : 2;
  __shared__ StatAcc<MODE> red[WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const bool cok = c < C;
  const int ny = ny1, by = blockIdx.y;
  auto finish = [&](StatAcc<MODE> t) {
    if constexpr (MODE == 0) {
      out[c] = t.b;
      out[C + c] = t.a > 0.f ? t.c / t.a : 0.f;
    } else {
      out[c] = t.a;
      out[C + c] = t.b;
    }
  };
  // ---- level 1: wave w merges rows [b0 + 16w, b0 + 16w + 16) of this block ----
  const int w0 = by * (WAVES * kStatRW) + w * kStatRW;
  red[w][lane] = cok ? stat_tree<MODE, kStatRW>(slab, (long)NV * C, w0, min(rows, w0 + kStatRW), C, c)
                     : StatAcc<MODE>::zero();
  stat_tree_lds<MODE, WAVES>(red, w, lane);
  if (ny == 1) {
    if (w == 0 && cok) finish(red[0][lane]);
    return;
  }
  // ny > 1: publish this block's partial; the consuming apply kernel merges the ny partials of
  // its channels in part order in its prologue (read_stats), so there is no second level here:
  // no ticket, no release/acquire fences, no serial last block (the kernel boundary publishes)
  if (w == 0 && cok) {
    const StatAcc<MODE> t = red[0][lane];
    part[((long)by * 3 + 0) * C + c] = t.a;
    part[((long)by * 3 + 1) * C + c] = t.b;
    part[((long)by * 3 + 2) * C + c] = t.c;
  }
}

// Statistics as the consumers see them: parts == 1 -> buf is the finished [2][C] result of
// bn_stat_reduce; parts > 1 -> buf holds its [parts][3][C] level-1 partials, merged here in part
// order (fixed: deterministic). MODE 0 -> (mean, biased variance), MODE 1 -> (sum a, sum b).
template <int MODE>
__device__ __forceinline__ void read_stats(const float* __restrict__ buf, int parts, int C, int c, float& s0,
                                           float& s1) {
  if (parts <= 1) {
    s0 = buf[c];
    s1 = buf[C + c];
    return;
  }
  StatAcc<MODE> t{buf[c], buf[C + c], buf[2 * C + c]};
  // four partials' loads in flight at once, merged in part order (same order as one at a time)
  int p = 1;
  for (; p + 3 < parts; p += 4) {
    StatAcc<MODE> q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* r = buf + (long)(p + u) * 3 * C + c;
      q[u] = StatAcc<MODE>{r[0], r[C], r[2 * C]};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) t = t.merge(q[u]);
  }
  for (; p < parts; ++p) {
    const float* q = buf + (long)p * 3 * C + c;
    t = t.merge(StatAcc<MODE>{q[0], q[C], q[2 * C]});
  }
  if constexpr (MODE == 0) {
    s0 = t.b;
    s1 = t.a > 0.f ? t.c / t.a : 0.f;
  } else {
    s0 = t.a;
    s1 = t.b;
  }
}

// y = x*scale + shift (+ residual) (ReLU); scale/shift from batch sums or running stats.
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, T* __restrict__ y, long R, int C,
                                                       const float* __restrict__ sums, int parts, float count,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       const T* __restrict__ residual, int relu,
                                                       float* __restrict__ save_mean, float* __restrict__ save_istd,
                                                       float* __restrict__ run_mean, float* __restrict__ run_var,
                                                       float momentum, int use_running) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* scale = sh;
  float* shift = sh + C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, istd;
    if (use_running) {
      mean = run_mean[c];
      istd = rsqrtf(run_var[c] + eps);
    } else {
      float var;
      read_stats<0>(sums, parts, C, c, mean, var);  // (mean, biased variance)
      istd = rsqrtf(var + eps);
      if (blockIdx.x == 0) {
        if (save_mean) { save_mean[c] = mean; save_istd[c] = istd; }
        if (run_mean) {
          const float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
          run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
          run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
        }
      }
    }
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    scale[c] = g * istd;
    shift[c] = b - mean * g * istd;
  }
  __syncthreads();
  const long nv = R * C / V;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x) {
    const long o = i * V;
    const int c0 = (int)(o % C);
    float xv[V];
    vload<T, V>(x + o, xv);
    float r[V];
    if (residual) vload<T, V>(residual + o, r);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float t = xv[v] * scale[c0 + v] + shift[c0 + v];
      if (residual) t += r[v];
      if (relu) t = fmaxf(t, 0.f);
      xv[v] = t;
    }
    vstore<T, V>(y + o, xv);
  }
}

// Training-mode BatchNorm + ReLU + non-overlapping max-pool in one pass (the ResNet stem):
// y[n][oy][ox][c] = max over the window of relu(x * scale + shift), rounded to bf16 BEFORE the
// comparison exactly as bn_apply + maxpool_fwd would, idx = window position of the max. The
// full-resolution BN output is never written: the backward (maxpool_bwd_bnb) masks with the
// pooled value and recomputes xhat from x.
// P > 0: a compile-time P x P window (the ResNet stems' 2 x 2): the window's loads are issued
// together instead of one dependent load per window pixel (the run-time loop serialised them)
template <int P>
__global__ void __launch_bounds__(256) bn_relu_maxpool_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                              uint8_t* __restrict__ idx, PoolGeom g,
                                                              const float* __restrict__ sums, int parts,
                                                              float count, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps,
                                                              float* __restrict__ save_mean,
                                                              float* __restrict__ save_istd,
                                                              float* __restrict__ run_mean,
                                                              float* __restrict__ run_var, float momentum) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* scale = sh;
  float* shift = sh + g.C;
  for (int c = threadIdx.x; c < g.C; c += blockDim.x) {
    float mean, var;
    read_stats<0>(sums, parts, g.C, c, mean, var);  // (mean, biased variance)
    const float istd = rsqrtf(var + eps);
    if (blockIdx.x == 0) {
      if (save_mean) { save_mean[c] = mean; save_istd[c] = istd; }
      if (run_mean) {
        const float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
      }
    }
    const float gm = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    scale[c] = gm * istd;
    shift[c] = b - mean * gm * istd;
  }
  __syncthreads();
  const int CV = g.C / 8;
  const long total = (long)g.N * g.OH * g.OW * CV;
  const bool small = total < (1l << 32);  // 32-bit index math (64-bit div/mod chains are ALU heavy)
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cv, ox, oy, n;
    if (small) {
      const unsigned iu = (unsigned)i;
      unsigned t = iu / (unsigned)CV;
      cv = (int)(iu - t * (unsigned)CV);
      ox = (int)(t % (unsigned)g.OW);
      t /= (unsigned)g.OW;
      oy = (int)(t % (unsigned)g.OH);
      n = (int)(t / (unsigned)g.OH);
    } else {
      cv = (int)(i % CV);
      long t = i / CV;
      ox = (int)(t % g.OW);
      t /= g.OW;
      oy = (int)(t % g.OH);
      n = (int)(t / g.OH);
    }
    float sc[8], sf[8], best[8], v[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = scale[cv * 8 + e]; sf[e] = shift[cv * 8 + e]; best[e] = -INFINITY; bi[e] = 0; }
    auto take = [&](const uint4& raw, int local) {
      unpack8(raw, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float r = (float)(bf16)fmaxf(v[e] * sc[e] + sf[e], 0.f);
        if (r > best[e]) { best[e] = r; bi[e] = (uint8_t)local; }
      }
    };
    if constexpr (P > 0) {
      uint4 w[P * P];
#pragma unroll
      for (int ky = 0; ky < P; ++ky)
#pragma unroll
        for (int kx = 0; kx < P; ++kx)
          w[ky * P + kx] = *reinterpret_cast<const uint4*>(
              x + (((long)n * g.H + oy * P + ky) * g.W + ox * P + kx) * g.C + cv * 8);
#pragma unroll
      for (int k = 0; k < P * P; ++k) take(w[k], k);
    } else {
      for (int ky = 0; ky < g.ph; ++ky)
        for (int kx = 0; kx < g.pw; ++kx) {
          const int iy = oy * g.ph + ky, ix = ox * g.pw + kx;
          take(*reinterpret_cast<const uint4*>(x + (((long)n * g.H + iy) * g.W + ix) * g.C + cv * 8), ky * g.pw + kx);
        }
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(best);
    *reinterpret_cast<uint2*>(idx + i * 8) = *reinterpret_cast<uint2*>(bi);
  }
}

// dx = gamma*istd*(dy' - sum_dy/M - xhat*sum_dyxhat/M); block 0 accumulates dgamma/dbeta.
template <typename T, int V>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ yout,
                                                           const T* __restrict__ x, T* __restrict__ dx, long R,
                                                           int C, const float* __restrict__ mean,
                                                           const float* __restrict__ istd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sums, int parts,
                                                           float count, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta, int eval_mode) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* ca = sh;          // gamma*istd
  float* cb = sh + C;      // mean(dy')
  float* cc = sh + 2 * C;  // mean(dy' xhat)
  float* cm = sh + 3 * C;  // mean
  float* ci = sh + 4 * C;  // istd
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float g = gamma ? gamma[c] : 1.f;
    float sdy = 0.f, sdyx = 0.f;
    if (sums) read_stats<1>(sums, parts, C, c, sdy, sdyx);
    ca[c] = g * istd[c];
    cb[c] = eval_mode ? 0.f : sdy / count;
    cc[c] = eval_mode ? 0.f : sdyx / count;
    cm[c] = mean[c];
    ci[c] = istd[c];
    if (blockIdx.x == 0 && sums) {
      if (dgamma) dgamma[c] += sdyx;
      if (dbeta) dbeta[c] += sdy;
    }
  }
  __syncthreads();
  const long nv = R * C / V;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x) {
    const long o = i * V;
    const int c0 = (int)(o % C);
    float d[V], xv[V];
    vload<T, V>(dy + o, d);
    vload<T, V>(x + o, xv);
    if (yout) {
      float yo[V];
      vload<T, V>(yout + o, yo);
#pragma unroll
      for (int v = 0; v < V; ++v) d[v] = yo[v] > 0.f ? d[v] : 0.f;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = c0 + v;
      const float xh = (xv[v] - cm[c]) * ci[c];
      d[v] = ca[c] * (d[v] - cb[c] - xh * cc[c]);
    }
    vstore<T, V>(dx + o, d);
  }
}

// ---------------------------------------------------------------------------------------
// bf16 apply passes at HBM speed (C % 8 == 0, fewer than 2^31 elements). The generic kernels
// above move one 16-byte vector per thread per trip with the per-channel prologue (a chain of
// statistics-partial merges) in front of the first load, so the short ResNet passes spent a
// large share of their time in that prologue and with one load in flight per lane. Here each
// thread owns U vectors per trip (all U loads issued together), its FIRST trip's loads are
// issued before the prologue (the prologue's latency hides behind them), channel coefficients
// come from LDS as float4s, and indexing is 32-bit.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 ldg16(const bf16* p) { return *reinterpret_cast<const uint4*>(p); }

// 8-element vectors of the apply passes: one 16-byte bf16 vector, or two 16-byte fp32 halves
// (the fp32 compute path; same trips / prologue scheme, twice the bytes per vector)
template <typename T>
struct Vec8;
template <>
struct Vec8<bf16> {
  using type = uint4;
  __device__ __forceinline__ static type load(const bf16* p) { return ldg16(p); }
  __device__ __forceinline__ static void unpack(const type& v, float* f) { unpack8(v, f); }
  __device__ __forceinline__ static void store(bf16* p, const float* f) { *reinterpret_cast<uint4*>(p) = pack8(f); }
};
template <>
struct Vec8<float> {
  struct type {
    float4 a, b;
  };
  __device__ __forceinline__ static type load(const float* p) {
    return type{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
  }
  __device__ __forceinline__ static void unpack(const type& v, float* f) {
    f[0] = v.a.x; f[1] = v.a.y; f[2] = v.a.z; f[3] = v.a.w;
    f[4] = v.b.x; f[5] = v.b.y; f[6] = v.b.z; f[7] = v.b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
};

// y = x*scale + shift (+ residual) (ReLU)
template <typename T, int U, bool RES>
__global__ void __launch_bounds__(256) bn_apply_v_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                         unsigned nv, int C, const float* __restrict__ sums,
                                                         int parts, float count, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps,
                                                         const T* __restrict__ residual, int relu,
                                                         float* __restrict__ save_mean,
                                                         float* __restrict__ save_istd,
                                                         float* __restrict__ run_mean, float* __restrict__ run_var,
                                                         float momentum, int use_running) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* scale = sh;
  float* shift = sh + C;
  using VT = Vec8<T>;
  const unsigned stride = gridDim.x * 256u, cv = (unsigned)C / 8;
  unsigned i = blockIdx.x * 256u + threadIdx.x;
  typename VT::type xv[U], rv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned k = i + u * stride;
    if (k < nv) {
      xv[u] = VT::load(x + (size_t)k * 8);
      if (RES) rv[u] = VT::load(residual + (size_t)k * 8);
    }
  }
  // the coefficient table, four channels per lane per round with all their loads issued together
  // (channel indices clamped so the loads need no guard; C = 2048 is 8 channels per lane)
  auto table = [&](auto j_c) {
    constexpr int J = decltype(j_c)::value;
    for (int cb = threadIdx.x; cb < C; cb += 256 * J) {
      float m4[J], v4[J], g4[J], b4[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = min(cb + 256 * j, C - 1);
        if (use_running) {
          m4[j] = run_mean[c];
          v4[j] = run_var[c];
        } else if (parts <= 1) {
          m4[j] = sums[c];
          v4[j] = sums[C + c];
        } else {
          read_stats<0>(sums, parts, C, c, m4[j], v4[j]);
        }
        g4[j] = gamma ? gamma[c] : 1.f;
        b4[j] = beta ? beta[c] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = cb + 256 * j;
        if (c >= C) break;
        const float mean = m4[j], var = v4[j], istd = rsqrtf(var + eps);
        if (!use_running && blockIdx.x == 0) {
          if (save_mean) { save_mean[c] = mean; save_istd[c] = istd; }
          if (run_mean) {
            const float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
            run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
            run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
          }
        }
        scale[c] = g4[j] * istd;
        shift[c] = b4[j] - mean * g4[j] * istd;
      }
    }
  };
  // (one channel per lane per round up to C = 256: the clamped extra loads cost the short passes)
  if (C > 256)
    table(std::integral_constant<int, 4>{});
  else
    table(std::integral_constant<int, 1>{});
  __syncthreads();
  while (true) {
    // the next trip's loads go out before this trip's stores (loads and stores overlap)
    const unsigned inx = i + U * stride;
    typename VT::type xn[U], rn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = inx + u * stride;
      if (inx < nv && k < nv) {
        xn[u] = VT::load(x + (size_t)k * 8);
        if (RES) rn[u] = VT::load(residual + (size_t)k * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = i + u * stride;
      if (k < nv) {
        const int c0 = (int)((cv & (cv - 1)) == 0 ? (k & (cv - 1)) : k % cv) * 8;  // (C / 8 a power of two: a mask)
        const float4 s0 = *reinterpret_cast<const float4*>(scale + c0), s1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(shift + c0), h1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sf[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        float f[8], r[8];
        VT::unpack(xv[u], f);
        if (RES) VT::unpack(rv[u], r);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          float t = f[v] * sc[v] + sf[v];
          if (RES) t += r[v];
          if (relu) t = fmaxf(t, 0.f);
          f[v] = t;
        }
        VT::store(y + (size_t)k * 8, f);
      }
    }
    if (inx >= nv) break;
    i = inx;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = xn[u];
      if (RES) rv[u] = rn[u];
    }
  }
}

// dx = A*dy' + B*(x - mean) + D per channel, with A = gamma*istd, B = -A*istd*mean(dy' xhat),
// D = -A*mean(dy') (the same algebra as bn_bwd_apply_kernel, three coefficients instead of five)
template <typename T, int U, bool MASK>
__global__ void __launch_bounds__(256) bn_bwd_apply_v_kernel(const T* __restrict__ dy,
                                                             const T* __restrict__ yout,
                                                             const T* __restrict__ x, T* __restrict__ dx,
                                                             unsigned nv, int C, const float* __restrict__ mean,
                                                             const float* __restrict__ istd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ sums, int parts, float count,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                             int eval_mode) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* ca = sh;          // A
  float* cbm = sh + C;     // B
  float* cm = sh + 2 * C;  // mean
  float* cd = sh + 3 * C;  // D
  using VT = Vec8<T>;
  const unsigned stride = gridDim.x * 256u, cv = (unsigned)C / 8;
  unsigned i = blockIdx.x * 256u + threadIdx.x;
  typename VT::type dv[U], xv[U], yv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned k = i + u * stride;
    if (k < nv) {
      dv[u] = VT::load(dy + (size_t)k * 8);
      xv[u] = VT::load(x + (size_t)k * 8);
      if (MASK) yv[u] = VT::load(yout + (size_t)k * 8);
    }
  }
  // (four channels per lane per round, loads together: as bn_apply_v_kernel)
  auto table = [&](auto j_c) {
    constexpr int J = decltype(j_c)::value;
    for (int cb = threadIdx.x; cb < C; cb += 256 * J) {
      float g4[J], is4[J], m4[J], s4[J], sx4[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = min(cb + 256 * j, C - 1);
        g4[j] = gamma ? gamma[c] : 1.f;
        is4[j] = istd[c];
        m4[j] = mean[c];
        s4[j] = 0.f;
        sx4[j] = 0.f;
        if (sums) {
          if (parts <= 1) {
            s4[j] = sums[c];
            sx4[j] = sums[C + c];
          } else {
            read_stats<1>(sums, parts, C, c, s4[j], sx4[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = cb + 256 * j;
        if (c >= C) break;
        const float is = is4[j], sdy = s4[j], sdyx = sx4[j];
        const float a = g4[j] * is;
        ca[c] = a;
        cbm[c] = eval_mode ? 0.f : -a * is * (sdyx / count);
        cm[c] = m4[j];
        cd[c] = eval_mode ? 0.f : -a * (sdy / count);
        if (blockIdx.x == 0 && sums) {
          if (dgamma) dgamma[c] += sdyx;
          if (dbeta) dbeta[c] += sdy;
        }
      }
    }
  };
  // (one channel per lane per round up to C = 256: the clamped extra loads cost the short passes)
  if (C > 256)
    table(std::integral_constant<int, 4>{});
  else
    table(std::integral_constant<int, 1>{});
  __syncthreads();
  auto ld8 = [](const float* p, float* o) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  };
  while (true) {
    const unsigned inx = i + U * stride;  // next trip's loads before this trip's stores
    typename VT::type dn[U], xn[U], yn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = inx + u * stride;
      if (inx < nv && k < nv) {
        dn[u] = VT::load(dy + (size_t)k * 8);
        xn[u] = VT::load(x + (size_t)k * 8);
        if (MASK) yn[u] = VT::load(yout + (size_t)k * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = i + u * stride;
      if (k < nv) {
        const int c0 = (int)((cv & (cv - 1)) == 0 ? (k & (cv - 1)) : k % cv) * 8;  // (C / 8 a power of two: a mask)
        float A[8], B[8], M[8], D[8], d[8], xf[8];
        ld8(ca + c0, A);
        ld8(cbm + c0, B);
        ld8(cm + c0, M);
        ld8(cd + c0, D);
        VT::unpack(dv[u], d);
        VT::unpack(xv[u], xf);
        if (MASK) {
          float yo[8];
          VT::unpack(yv[u], yo);
#pragma unroll
          for (int v = 0; v < 8; ++v) d[v] = yo[v] > 0.f ? d[v] : 0.f;
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) d[v] = A[v] * d[v] + B[v] * (xf[v] - M[v]) + D[v];
        VT::store(dx + (size_t)k * 8, d);
      }
    }
    if (inx >= nv) break;
    i = inx;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dv[u] = dn[u];
      xv[u] = xn[u];
      if (MASK) yv[u] = yn[u];
    }
  }
}

// y = act(a.x * sa + ha + b.x * sb + hb): the tail BatchNorm of a residual block and its
// projection shortcut's BatchNorm in one pass (the shortcut's normalised output is never
// written or re-read). Same trips / prologue scheme as bn_apply_v_kernel; workgroup 0 saves both
// layers' (mean, istd) and updates both running statistics.
__device__ __forceinline__ void bn_side_coeffs(const BnSide& b, int C, float* scale, float* shift, bool first) {
  // (four channels per lane per round, loads together: as bn_apply_v_kernel)
  auto table = [&](auto j_c) {
    constexpr int J = decltype(j_c)::value;
    for (int cb = threadIdx.x; cb < C; cb += 256 * J) {
      float m4[J], v4[J], g4[J], b4[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = min(cb + 256 * j, C - 1);
        if (b.use_running) {
          m4[j] = b.run_mean[c];
          v4[j] = b.run_var[c];
        } else if (b.parts <= 1) {
          m4[j] = b.sums[c];
          v4[j] = b.sums[C + c];
        } else {
          read_stats<0>(b.sums, b.parts, C, c, m4[j], v4[j]);
        }
        g4[j] = b.gamma ? b.gamma[c] : 1.f;
        b4[j] = b.beta ? b.beta[c] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = cb + 256 * j;
        if (c >= C) break;
        const float mean = m4[j], var = v4[j], istd = rsqrtf(var + b.eps);
        if (!b.use_running && first) {
          if (b.save_mean) { b.save_mean[c] = mean; b.save_istd[c] = istd; }
          if (b.run_mean) {
            const float unbiased = b.count > 1.f ? var * b.count / (b.count - 1.f) : var;
            b.run_mean[c] = (1.f - b.momentum) * b.run_mean[c] + b.momentum * mean;
            b.run_var[c] = (1.f - b.momentum) * b.run_var[c] + b.momentum * unbiased;
          }
        }
        scale[c] = g4[j] * istd;
        shift[c] = b4[j] - mean * g4[j] * istd;
      }
    }
  };
  // (one channel per lane per round up to C = 256: the clamped extra loads cost the short passes)
  if (C > 256)
    table(std::integral_constant<int, 4>{});
  else
    table(std::integral_constant<int, 1>{});
}

__global__ void __launch_bounds__(256) bn_apply_dual_kernel(BnSide a, BnSide b, bf16* __restrict__ y, unsigned nv,
                                                            int C, int relu) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* sa = sh;
  float* ha = sh + C;
  float* sb = sh + 2 * C;
  float* hb = sh + 3 * C;
  const bf16* __restrict__ xa = static_cast<const bf16*>(a.x);
  const bf16* __restrict__ xb = static_cast<const bf16*>(b.x);
  const unsigned stride = gridDim.x * 256u, cv = (unsigned)C / 8;
  unsigned i = blockIdx.x * 256u + threadIdx.x;
  uint4 va{}, vb{};
  if (i < nv) {
    va = ldg16(xa + (size_t)i * 8);
    vb = ldg16(xb + (size_t)i * 8);
  }
  bn_side_coeffs(a, C, sa, ha, blockIdx.x == 0);
  bn_side_coeffs(b, C, sb, hb, blockIdx.x == 0);
  __syncthreads();
  auto ld8 = [](const float* p, float* o) {
    const float4 u = *reinterpret_cast<const float4*>(p), v = *reinterpret_cast<const float4*>(p + 4);
    o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
  };
  while (i < nv) {
    const unsigned inx = i + stride;  // next trip's loads before this trip's store
    uint4 na{}, nb{};
    if (inx < nv) {
      na = ldg16(xa + (size_t)inx * 8);
      nb = ldg16(xb + (size_t)inx * 8);
    }
    const int c0 = (int)((cv & (cv - 1)) == 0 ? (i & (cv - 1)) : i % cv) * 8;  // (C / 8 a power of two: a mask)
    float A[8], HA[8], B[8], HB[8], fa[8], fb[8];
    ld8(sa + c0, A);
    ld8(ha + c0, HA);
    ld8(sb + c0, B);
    ld8(hb + c0, HB);
    unpack8(va, fa);
    unpack8(vb, fb);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float t = fa[v] * A[v] + HA[v];
      // the shortcut branch rounded to bf16 as the materialised shortcut tensor would be
      t += (float)(bf16)(fb[v] * B[v] + HB[v]);
      if (relu) t = fmaxf(t, 0.f);
      fa[v] = t;
    }
    *reinterpret_cast<uint4*>(y + (size_t)i * 8) = pack8(fa);
    i = inx;
    va = na;
    vb = nb;
  }
}

// (the dual backward stages 8 coefficient arrays of C floats in dynamic LDS: 32*C bytes must fit
// the 64 KB a launch gets without a raised limit, i.e. C <= 2048; wider layers use the separate
// per-side passes)
bool bn_apply_dual_supported(long R, int C) {
  return C % 8 == 0 && 8L * C * (long)sizeof(float) <= 65536 && R * (long)C < (1l << 31);
}

// Backward of two BatchNorms fed the same gradient dy (a residual block's tail and its projection
// shortcut): dx_a and dx_b from one read of dy, each side with bn_bwd_apply_v_kernel's
// 3-coefficient algebra (identical per-element results) and workgroup 0 accumulating its dgamma
// / dbeta.
__device__ __forceinline__ void bn_bwd_side_coeffs(const BnBwdSide& b, int C, float* ca, float* cbm, float* cm,
                                                   float* cd, bool first) {
  // (four channels per lane per round, loads together: as bn_apply_v_kernel)
  auto table = [&](auto j_c) {
    constexpr int J = decltype(j_c)::value;
    for (int cb = threadIdx.x; cb < C; cb += 256 * J) {
      float g4[J], is4[J], m4[J], s4[J], sx4[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = min(cb + 256 * j, C - 1);
        g4[j] = b.gamma ? b.gamma[c] : 1.f;
        is4[j] = b.istd[c];
        m4[j] = b.mean[c];
        s4[j] = 0.f;
        sx4[j] = 0.f;
        if (b.sums) {
          if (b.parts <= 1) {
            s4[j] = b.sums[c];
            sx4[j] = b.sums[C + c];
          } else {
            read_stats<1>(b.sums, b.parts, C, c, s4[j], sx4[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = cb + 256 * j;
        if (c >= C) break;
        const float is = is4[j], sdy = s4[j], sdyx = sx4[j];
        const float a = g4[j] * is;
        ca[c] = a;
        cbm[c] = -a * is * (sdyx / b.count);
        cm[c] = m4[j];
        cd[c] = -a * (sdy / b.count);
        if (first && b.sums) {
          if (b.dgamma) b.dgamma[c] += sdyx;
          if (b.dbeta) b.dbeta[c] += sdy;
        }
      }
    }
  };
  // (one channel per lane per round up to C = 256: the clamped extra loads cost the short passes)
  if (C > 256)
    table(std::integral_constant<int, 4>{});
  else
    table(std::integral_constant<int, 1>{});
}

__global__ void __launch_bounds__(256) bn_bwd_apply_dual_kernel(const bf16* __restrict__ dy, BnBwdSide a,
                                                                BnBwdSide b, unsigned nv, int C) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* k = sh;  // [2 sides][4 coefficient arrays][C]
  const bf16* __restrict__ xa = static_cast<const bf16*>(a.x);
  const bf16* __restrict__ xb = static_cast<const bf16*>(b.x);
  bf16* __restrict__ da = static_cast<bf16*>(a.dx);
  bf16* __restrict__ db = static_cast<bf16*>(b.dx);
  const unsigned stride = gridDim.x * 256u, cv = (unsigned)C / 8;
  unsigned i = blockIdx.x * 256u + threadIdx.x;
  uint4 vd{}, va{}, vb{};
  if (i < nv) {
    vd = ldg16(dy + (size_t)i * 8);
    va = ldg16(xa + (size_t)i * 8);
    vb = ldg16(xb + (size_t)i * 8);
  }
  bn_bwd_side_coeffs(a, C, k, k + C, k + 2 * C, k + 3 * C, blockIdx.x == 0);
  bn_bwd_side_coeffs(b, C, k + 4 * C, k + 5 * C, k + 6 * C, k + 7 * C, blockIdx.x == 0);
  __syncthreads();
  auto ld8 = [](const float* p, float* o) {
    const float4 u = *reinterpret_cast<const float4*>(p), v = *reinterpret_cast<const float4*>(p + 4);
    o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
  };
  while (i < nv) {
    const unsigned inx = i + stride;
    uint4 nd{}, na{}, nb{};
    if (inx < nv) {
      nd = ldg16(dy + (size_t)inx * 8);
      na = ldg16(xa + (size_t)inx * 8);
      nb = ldg16(xb + (size_t)inx * 8);
    }
    const int c0 = (int)((cv & (cv - 1)) == 0 ? (i & (cv - 1)) : i % cv) * 8;  // (C / 8 a power of two: a mask)
    float d[8];
    unpack8(vd, d);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const float* ks = k + side * 4 * C;
      float A[8], B[8], M[8], D[8], xf[8], o[8];
      ld8(ks + c0, A);
      ld8(ks + C + c0, B);
      ld8(ks + 2 * C + c0, M);
      ld8(ks + 3 * C + c0, D);
      unpack8(side == 0 ? va : vb, xf);
#pragma unroll
      for (int v = 0; v < 8; ++v) o[v] = A[v] * d[v] + B[v] * (xf[v] - M[v]) + D[v];
      *reinterpret_cast<uint4*>((side == 0 ? da : db) + (size_t)i * 8) = pack8(o);
    }
    i = inx;
    vd = nd;
    va = na;
    vb = nb;
  }
}

bool bn_bwd_apply_dual(const void* dy, const BnBwdSide& a, const BnBwdSide& b, long R, int C, hipStream_t s) {
  if (!bn_apply_dual_supported(R, C)) return false;
  const unsigned nv = (unsigned)(R * C / 8);
  long g = (nv + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, dim3((unsigned)g), dim3(256), 8 * C * sizeof(float), s,
                     static_cast<const bf16*>(dy), a, b, nv, C);
  DCNN_LAUNCH_CHECK();
  return true;
}



bool bn_apply_dual(const BnSide& a, const BnSide& b, void* y, long R, int C, int relu, hipStream_t s) {
  if (!bn_apply_dual_supported(R, C)) return false;
  const unsigned nv = (unsigned)(R * C / 8);
  long g = (nv + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(bn_apply_dual_kernel, dim3((unsigned)g), dim3(256), 4 * C * sizeof(float), s, a, b,
                     static_cast<bf16*>(y), nv, C, relu);
  DCNN_LAUNCH_CHECK();
  return true;
}

// vectors per thread per trip and grid of the bf16 apply passes
static void bn_v_launch_shape(long nv, int C, int* U, int* grid) {
  // default: 1 vector per lane per trip, at most 1024 workgroups, so the large passes make
  // several software-pipelined trips (next trip's loads in flight under this trip's stores).
  // Measured on the ResNet-18 shapes (benchmarks/bn_bench.py, tools/gpu_bnsweep.sh): one pass
  // over all 12 shape/op cases 117.9 us with 4 vectors per lane over <= 2048 workgroups ->
  // 107.7 us (2 vectors: 107.0 us, but 0.5% slower end to end at batch 64 / 128)
  constexpr long g_cap = 1024;
  *U = 1;
  (void)C;  // (fewer, wider workgroups for C >= 1024 measured slower: profiles/bn_bandwidth_r6.md)
  const long cap = g_cap;
  long g = (nv + 256l * *U - 1) / (256l * *U);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  *grid = (int)g;
}

static bool g_bn_v = true;  // bn_set_vectorised(0): the generic kernels (test hook)

void bn_set_vectorised(int on) { g_bn_v = on != 0; }

static bool bn_v_ok(long R, int C) { return g_bn_v && C % 8 == 0 && R * (long)C < (1l << 31); }

// ---------------------------------------------------------------------------------------
// GroupNorm (NHWC): one workgroup per (image, group)
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) gn_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int HW, int C,
                                                     int G, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     float* __restrict__ save_mean, float* __restrict__ save_istd) {
  __shared__ float sh[16];
  const int n = blockIdx.x / G, g = blockIdx.x % G, Cg = C / G;
  const long base = (long)n * HW * C + (long)g * Cg;
  const long cnt = (long)HW * Cg;
  float s = 0.f;
  for (long i = threadIdx.x; i < cnt; i += blockDim.x) s += to_f(x[base + (i / Cg) * C + (i % Cg)]);
  const float mean = block_sum(s, sh) / (float)cnt;
  float q = 0.f;
  for (long i = threadIdx.x; i < cnt; i += blockDim.x) {
    const float d = to_f(x[base + (i / Cg) * C + (i % Cg)]) - mean;
    q += d * d;
  }
  __syncthreads();
  const float var = block_sum(q, sh) / (float)cnt;
  const float is = rsqrtf(var + eps);
  if (threadIdx.x == 0) { save_mean[blockIdx.x] = mean; save_istd[blockIdx.x] = is; }
  for (long i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int c = g * Cg + (int)(i % Cg);
    const long o = base + (i / Cg) * C + (i % Cg);
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    y[o] = from_f<T>((to_f(x[o]) - mean) * is * gm + bt);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gn_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     T* __restrict__ dx, int HW, int C, int G,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ istd,
                                                     float* __restrict__ aff) {
  __shared__ float sh[16];
  const int n = blockIdx.x / G, g = blockIdx.x % G, Cg = C / G;
  const long base = (long)n * HW * C + (long)g * Cg;
  const long cnt = (long)HW * Cg;
  const float mu = mean[blockIdx.x], is = istd[blockIdx.x];
  float s1 = 0.f, s2 = 0.f;
  for (long i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int c = g * Cg + (int)(i % Cg);
    const long o = base + (i / Cg) * C + (i % Cg);
    const float gm = gamma ? gamma[c] : 1.f;
    const float d = to_f(dy[o]) * gm, xh = (to_f(x[o]) - mu) * is;
    s1 += d;
    s2 += d * xh;
  }
  const float m1 = block_sum(s1, sh) / (float)cnt;
  __syncthreads();
  const float m2 = block_sum(s2, sh) / (float)cnt;
  for (long i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int c = g * Cg + (int)(i % Cg);
    const long o = base + (i / Cg) * C + (i % Cg);
    const float gm = gamma ? gamma[c] : 1.f;
    const float d = to_f(dy[o]) * gm, xh = (to_f(x[o]) - mu) * is;
    dx[o] = from_f<T>(is * (d - m1 - xh * m2));
  }
  // per-channel dgamma/dbeta partial of this image -> aff[n][2][C] (summed over images in a fixed
  // order by gn_affine_reduce_kernel: no float atomics)
  for (int cl = threadIdx.x; cl < Cg; cl += blockDim.x) {
    const int c = g * Cg + cl;
    float a = 0.f, b = 0.f;
    for (int p = 0; p < HW; ++p) {
      const long o = base + (long)p * C + cl;
      const float d = to_f(dy[o]);
      a += d * (to_f(x[o]) - mu) * is;
      b += d;
    }
    aff[((long)n * 2 + 0) * C + c] = a;
    aff[((long)n * 2 + 1) * C + c] = b;
  }
}

__global__ void gn_affine_reduce_kernel(const float* __restrict__ aff, int N, int C, float* __restrict__ dgamma,
                                        float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int n = 0; n < N; ++n) { a += aff[((long)n * 2 + 0) * C + c]; b += aff[((long)n * 2 + 1) * C + c]; }
  if (dgamma) dgamma[c] += a;
  if (dbeta) dbeta[c] += b;
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
static int bn_rows_per_block(long R, int C) {
  // ~ (256 CUs x 2) workgroups, each a multiple of the concurrent rows
  long rpb = (R + 511) / 512;
  if (rpb < 16) rpb = 16;
  return (int)rpb;
}

int bn_partial_rows(long R, int C) {
  const int rpb = bn_rows_per_block(R, C);
  return (int)((R + rpb - 1) / rpb);
}

template <typename T>
static void bn_partial_t(const T* x, const T* dy, const T* yout, T* dy_out, const float* mean,
                         const float* istd, long R, int C, float* slab, int mode, float* zs, hipStream_t s) {
  const int rpb = bn_rows_per_block(R, C);
  const int blocks = (int)((R + rpb - 1) / rpb);
  if (C % 8 == 0) {
    const int groups = C / 8, tpr = groups < 256 ? groups : 256, rc = 256 / tpr;
    const size_t shm = ((size_t)rc * 2 + 1) * tpr * 8 * sizeof(float);
    hipLaunchKernelGGL((bn_partial_kernel<T, 8>), dim3(blocks), dim3(256), shm, s, x, dy, yout, dy_out, mean,
                       istd, R, C, rpb, slab, mode, zs);
  } else {
    const int tpr = C < 256 ? C : 256, rc = 256 / tpr;
    const size_t shm = ((size_t)rc * 2 + 1) * tpr * sizeof(float);
    hipLaunchKernelGGL((bn_partial_kernel<T, 1>), dim3(blocks), dim3(256), shm, s, x, dy, yout, dy_out, mean,
                       istd, R, C, rpb, slab, mode, zs);
  }
  DCNN_LAUNCH_CHECK();
}

void bn_partial(int dtype, const void* x, const void* dy, const void* yout, void* dy_out, const float* mean,
                const float* istd, long R, int C, float* slab, int mode, float* zero_sums, hipStream_t s) {
  if (dtype == 0)
    bn_partial_t<float>((const float*)x, (const float*)dy, (const float*)yout, (float*)dy_out, mean, istd, R, C,
                        slab, mode, zero_sums, s);
  else
    bn_partial_t<bf16>((const bf16*)x, (const bf16*)dy, (const bf16*)yout, (bf16*)dy_out, mean, istd, R, C, slab,
                       mode, zero_sums, s);
}

int bn_stat_parts(int rows) {
  const int per = g_stat_waves * kStatRW;
  return (rows + per - 1) / per;
}

// mode 0: slab [rows][3][C] Welford triples -> out = (mean, var); mode 1: slab [rows][2][C] sums.
// part: bn_stat_parts(rows) x 3 x C floats (unused when that is 1); ticket: ceil(C/64) zeroed
// words, left zeroed again (one ticket array per stream).
void bn_stat_reduce2(int mode, const float* slab, int rows, float* out, float* part, const float* slab2, int rows2,
                     float* out2, float* part2, int C, hipStream_t s) {
  const int ny = bn_stat_parts(rows), ny2 = slab2 ? bn_stat_parts(rows2) : 0;
  if ((ny > 1 && !part) || (ny2 > 1 && !part2)) throw std::runtime_error("bn_stat_reduce: partials buffer required");
  const dim3 grid((unsigned)((C + 63) / 64), (unsigned)(ny > ny2 ? ny : ny2), slab2 ? 2u : 1u);
#define DCNN_SR(W)                                                                                           \
  if (g_stat_waves == W) {                                                                                   \
    if (mode == 0)                                                                                           \
      hipLaunchKernelGGL((bn_stat_reduce_kernel<0, W>), grid, dim3(64 * W), 0, s, slab, rows, C, part, nullptr, out, \
                         ny, slab2, rows2, part2, out2, ny2);                                                \
    else                                                                                                     \
      hipLaunchKernelGGL((bn_stat_reduce_kernel<1, W>), grid, dim3(64 * W), 0, s, slab, rows, C, part, nullptr, out, \
                         ny, slab2, rows2, part2, out2, ny2);                                                \
  }
  DCNN_SR(4) DCNN_SR(8) DCNN_SR(16)
#undef DCNN_SR
  DCNN_LAUNCH_CHECK();
}

void bn_stat_reduce(int mode, const float* slab, int rows, int C, float* out, float* part, unsigned* ticket,
                    hipStream_t s) {
  (void)ticket;  // (the in-kernel second level is gone: consumers merge the partials)
  bn_stat_reduce2(mode, slab, rows, out, part, nullptr, 0, nullptr, nullptr, C, s);
}

bool bn_relu_maxpool_supported(PoolGeom g) {
  return g.C % 8 == 0 && g.ph == g.sh && g.pw == g.sw && g.padh == 0 && g.padw == 0 && g.ph * g.pw <= 255 &&
         g.OH == g.H / g.ph && g.OW == g.W / g.pw;
}

void bn_relu_maxpool(const bf16* x, bf16* y, uint8_t* idx, PoolGeom g, const float* sums, int parts, float count,
                     const float* gamma, const float* beta, float eps, float* save_mean, float* save_istd,
                     float* run_mean, float* run_var, float momentum, hipStream_t s) {
  if (!bn_relu_maxpool_supported(g)) throw std::runtime_error("bn_relu_maxpool: unsupported geometry");
  const long total = (long)g.N * g.OH * g.OW * g.C / 8;
  auto k = (g.ph == 2 && g.pw == 2) ? bn_relu_maxpool_kernel<2> : bn_relu_maxpool_kernel<0>;
  hipLaunchKernelGGL(k, dim3(grid_for(total, 256, 2048)), dim3(256), 2 * g.C * sizeof(float), s,
                     x, y, idx, g, sums, parts, count, gamma, beta, eps, save_mean, save_istd, run_mean, run_var,
                     momentum);
  DCNN_LAUNCH_CHECK();
}

template <typename T>
static void bn_apply_t(const T* x, T* y, long R, int C, const float* sums, int parts, float count, const float* gamma,
                       const float* beta, float eps, const T* residual, int relu, float* save_mean,
                       float* save_istd, float* run_mean, float* run_var, float momentum, int use_running,
                       hipStream_t s) {
  const size_t shm = 2 * C * sizeof(float);
  if (bn_v_ok(R, C)) {
    int U, g;
    const unsigned nv = (unsigned)(R * C / 8);
    bn_v_launch_shape(nv, C, &U, &g);
#define DCNN_BNV(U_, RES_)                                                                                       \
  if (U == U_ && (residual != nullptr) == RES_)                                                                  \
    hipLaunchKernelGGL((bn_apply_v_kernel<T, U_, RES_>), dim3(g), dim3(256), shm, s, x, y, nv, C, sums, parts, count, \
                       gamma, beta, eps, residual, relu, save_mean, save_istd, run_mean, run_var, momentum, use_running);
    DCNN_BNV(1, false) DCNN_BNV(2, false) DCNN_BNV(4, false) DCNN_BNV(1, true) DCNN_BNV(2, true) DCNN_BNV(4, true)
#undef DCNN_BNV
    DCNN_LAUNCH_CHECK();
    return;
  }
  if (C % 8 == 0) {
    const int g = grid_for(R * C / 8, 256, 2048);
    hipLaunchKernelGGL((bn_apply_kernel<T, 8>), dim3(g), dim3(256), shm, s, x, y, R, C, sums, parts, count, gamma, beta,
                       eps, residual, relu, save_mean, save_istd, run_mean, run_var, momentum, use_running);
  } else {
    const int g = grid_for(R * C, 256, 2048);
    hipLaunchKernelGGL((bn_apply_kernel<T, 1>), dim3(g), dim3(256), shm, s, x, y, R, C, sums, parts, count, gamma, beta,
                       eps, residual, relu, save_mean, save_istd, run_mean, run_var, momentum, use_running);
  }
  DCNN_LAUNCH_CHECK();
}

void bn_apply(int dtype, const void* x, void* y, long R, int C, const float* sums, int parts, float count,
              const float* gamma, const float* beta, float eps, const void* residual, int relu, float* save_mean,
              float* save_istd, float* run_mean, float* run_var, float momentum, int use_running, hipStream_t s) {
  if (dtype == 0)
    bn_apply_t<float>((const float*)x, (float*)y, R, C, sums, parts, count, gamma, beta, eps, (const float*)residual,
                      relu, save_mean, save_istd, run_mean, run_var, momentum, use_running, s);
  else
    bn_apply_t<bf16>((const bf16*)x, (bf16*)y, R, C, sums, parts, count, gamma, beta, eps, (const bf16*)residual,
                     relu, save_mean, save_istd, run_mean, run_var, momentum, use_running, s);
}

template <typename T>
static void bn_bwd_apply_t(const T* dy, const T* yout, const T* x, T* dx, long R, int C, const float* mean,
                           const float* istd, const float* gamma, const float* sums, int parts, float count,
                           float* dgamma, float* dbeta, int eval_mode, hipStream_t s) {
  if (bn_v_ok(R, C)) {
    int U, g;
    const unsigned nv = (unsigned)(R * C / 8);
    bn_v_launch_shape(nv, C, &U, &g);
    const size_t shm4 = 4 * C * sizeof(float);
#define DCNN_BNBV(U_, MASK_)                                                                                      \
  if (U == U_ && (yout != nullptr) == MASK_)                                                                      \
    hipLaunchKernelGGL((bn_bwd_apply_v_kernel<T, U_, MASK_>), dim3(g), dim3(256), shm4, s, dy, yout, x, dx, nv, C, mean, \
                       istd, gamma, sums, parts, count, dgamma, dbeta, eval_mode);
    DCNN_BNBV(1, false) DCNN_BNBV(2, false) DCNN_BNBV(4, false) DCNN_BNBV(1, true) DCNN_BNBV(2, true) DCNN_BNBV(4, true)
#undef DCNN_BNBV
    DCNN_LAUNCH_CHECK();
    return;
  }
  const size_t shm = 5 * C * sizeof(float);
  if (C % 8 == 0) {
    const int g = grid_for(R * C / 8, 256, 2048);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, 8>), dim3(g), dim3(256), shm, s, dy, yout, x, dx, R, C, mean, istd,
                       gamma, sums, parts, count, dgamma, dbeta, eval_mode);
  } else {
    const int g = grid_for(R * C, 256, 2048);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, 1>), dim3(g), dim3(256), shm, s, dy, yout, x, dx, R, C, mean, istd,
                       gamma, sums, parts, count, dgamma, dbeta, eval_mode);
  }
  DCNN_LAUNCH_CHECK();
}

void bn_bwd_apply(int dtype, const void* dy, const void* yout, const void* x, void* dx, long R, int C,
                  const float* mean, const float* istd, const float* gamma, const float* sums, int parts, float count,
                  float* dgamma, float* dbeta, int eval_mode, hipStream_t s) {
  if (dtype == 0)
    bn_bwd_apply_t<float>((const float*)dy, (const float*)yout, (const float*)x, (float*)dx, R, C, mean, istd, gamma,
                          sums, parts, count, dgamma, dbeta, eval_mode, s);
  else
    bn_bwd_apply_t<bf16>((const bf16*)dy, (const bf16*)yout, (const bf16*)x, (bf16*)dx, R, C, mean, istd, gamma,
                         sums, parts, count, dgamma, dbeta, eval_mode, s);
}

void gn_fwd(int dtype, const void* x, void* y, int N, int HW, int C, int G, const float* gamma, const float* beta,
            float eps, float* save_mean, float* save_istd, hipStream_t s) {
  if (dtype == 0)
    hipLaunchKernelGGL(gn_fwd_kernel<float>, dim3(N * G), dim3(256), 0, s, (const float*)x, (float*)y, HW, C, G,
                       gamma, beta, eps, save_mean, save_istd);
  else
    hipLaunchKernelGGL(gn_fwd_kernel<bf16>, dim3(N * G), dim3(256), 0, s, (const bf16*)x, (bf16*)y, HW, C, G, gamma,
                       beta, eps, save_mean, save_istd);
  DCNN_LAUNCH_CHECK();
}

void gn_bwd(int dtype, const void* dy, const void* x, void* dx, int N, int HW, int C, int G, const float* gamma,
            const float* mean, const float* istd, float* dgamma, float* dbeta, float* aff, hipStream_t s) {
  if (dtype == 0)
    hipLaunchKernelGGL(gn_bwd_kernel<float>, dim3(N * G), dim3(256), 0, s, (const float*)dy, (const float*)x,
                       (float*)dx, HW, C, G, gamma, mean, istd, aff);
  else
    hipLaunchKernelGGL(gn_bwd_kernel<bf16>, dim3(N * G), dim3(256), 0, s, (const bf16*)dy, (const bf16*)x,
                       (bf16*)dx, HW, C, G, gamma, mean, istd, aff);
  DCNN_LAUNCH_CHECK();
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(gn_affine_reduce_kernel, dim3((C + 255) / 256), dim3(256), 0, s, aff, N, C, dgamma, dbeta);
    DCNN_LAUNCH_CHECK();
  }
}

}  // namespace dcnn
