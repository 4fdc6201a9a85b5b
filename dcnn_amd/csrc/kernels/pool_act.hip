// Pooling, activations, dropout, layout conversion and misc tensor kernels (NHWC, wave64).
//
// Reference kernels replaced: K29-K32 (src/nn/layers_impl/cuda/{maxpool,avgpool}_ops.cu: size_t
// argmax + atomicAdd scatter backward), K33 dropout (stored mask), K34-K36 activations,
// K12/K13 im2col/col2im (src/tensor/cuda/tensor_kernels.cu), K7/K8 transposes.
// Here: max-pool keeps a 1-byte window-local argmax and both pools use a GATHER backward
// (no atomics, deterministic, works for overlapping windows); dropout regenerates its
// Philox mask in backward (no mask tensor); activations are one templated elementwise kernel.
#include "common.h"
#include "api.h"

namespace dcnn {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i) { return to_f(p[i]); }

// ----------------------------------- pooling ---------------------------------------------


template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, PoolGeom g) {
  const long total = (long)g.N * g.OH * g.OW * g.C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    long t = i / g.C;
    const int ox = (int)(t % g.OW);
    t /= g.OW;
    const int oy = (int)(t % g.OH);
    const int n = (int)(t / g.OH);
    float best = -INFINITY;
    int bi = 0;
    for (int ky = 0; ky < g.ph; ++ky) {
      const int iy = oy * g.sh - g.padh + ky;
      if (iy < 0 || iy >= g.H) continue;
      for (int kx = 0; kx < g.pw; ++kx) {
        const int ix = ox * g.sw - g.padw + kx;
        if (ix < 0 || ix >= g.W) continue;
        const float v = ld(x, (((long)n * g.H + iy) * g.W + ix) * g.C + c);
        if (v > best) { best = v; bi = ky * g.pw + kx; }
      }
    }
    y[i] = from_f<T>(best);
    idx[i] = (uint8_t)bi;
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                   PoolGeom g) {
  const long total = (long)g.N * g.H * g.W * g.C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    long t = i / g.C;
    const int ix = (int)(t % g.W);
    t /= g.W;
    const int iy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    // windows containing (iy, ix): oy*sh - padh <= iy <= oy*sh - padh + ph - 1
    const int oy0 = max(0, (iy + g.padh - g.ph + g.sh) / g.sh), oy1 = min(g.OH - 1, (iy + g.padh) / g.sh);
    const int ox0 = max(0, (ix + g.padw - g.pw + g.sw) / g.sw), ox1 = min(g.OW - 1, (ix + g.padw) / g.sw);
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = iy - (oy * g.sh - g.padh);
      if (ky < 0 || ky >= g.ph) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = ix - (ox * g.sw - g.padw);
        if (kx < 0 || kx >= g.pw) continue;
        const long o = (((long)n * g.OH + oy) * g.OW + ox) * g.C + c;
        if (idx[o] == ky * g.pw + kx) acc += ld(dy, o);
      }
    }
    dx[i] = from_f<T>(acc);
  }
}

// Non-overlapping windows (stride == pool, no padding), bf16, 8 channels per thread:
// one 16-B load per window tap, one 8-B argmax store; the backward is a pure gather.
__global__ void maxpool_fwd_nov8_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, uint8_t* __restrict__ idx,
                                        PoolGeom g) {
  const int CV = g.C / 8;
  const long total = (long)g.N * g.OH * g.OW * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long t = i / CV;
    const int ox = (int)(t % g.OW);
    t /= g.OW;
    const int oy = (int)(t % g.OH);
    const int n = (int)(t / g.OH);
    float best[8], v[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int ky = 0; ky < g.ph; ++ky)
      for (int kx = 0; kx < g.pw; ++kx) {
        const int iy = oy * g.ph + ky, ix = ox * g.pw + kx;
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * g.H + iy) * g.W + ix) * g.C + cv * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(ky * g.pw + kx); }
      }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(best);
    *reinterpret_cast<uint2*>(idx + i * 8) = *reinterpret_cast<uint2*>(bi);
  }
}

__global__ void maxpool_bwd_nov8_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                        bf16* __restrict__ dx, PoolGeom g) {
  const int CV = g.C / 8;
  const long total = (long)g.N * g.H * g.W * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    long t = i / CV;
    const int ix = (int)(t % g.W);
    t /= g.W;
    const int iy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    const int oy = iy / g.ph, ox = ix / g.pw;
    float out[8];
    if (oy < g.OH && ox < g.OW) {
      const long o = (((long)n * g.OH + oy) * g.OW + ox) * g.C + cv * 8;
      const int local = (iy - oy * g.ph) * g.pw + (ix - ox * g.pw);
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + o), d);
      const uint2 ib = *reinterpret_cast<const uint2*>(idx + o);
      const uint8_t* b = reinterpret_cast<const uint8_t*>(&ib);
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = b[e] == local ? d[e] : 0.f;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = 0.f;
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(out);
  }
}

// The same for fp32 (the exact / split-precision fp32 paths): 4 channels per thread, one 16-B load
// per window tap, one 4-B argmax store, 32-bit index math (the generic per-element kernels spend
// their time in 64-bit div / mod chains: ResNet-9 fp32 max-pool backward 54 us per call).
__global__ void __launch_bounds__(256) maxpool_fwd_nov4f_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                uint8_t* __restrict__ idx, PoolGeom g) {
  const int CV = g.C >> 2;
  const int total = g.N * g.OH * g.OW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int t = i / CV;
    const int ox = t % g.OW;
    t /= g.OW;
    const int oy = t % g.OH, n = t / g.OH;
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint8_t bi[4] = {0, 0, 0, 0};
    for (int ky = 0; ky < g.ph; ++ky)
      for (int kx = 0; kx < g.pw; ++kx) {
        const int iy = oy * g.ph + ky, ix = ox * g.pw + kx;
        const float4 v4 = *reinterpret_cast<const float4*>(x + ((size_t)(n * g.H + iy) * g.W + ix) * g.C + cv * 4);
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(ky * g.pw + kx); }
      }
    *reinterpret_cast<float4*>(y + (size_t)i * 4) = make_float4(best[0], best[1], best[2], best[3]);
    *reinterpret_cast<uint32_t*>(idx + (size_t)i * 4) = *reinterpret_cast<const uint32_t*>(bi);
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_nov4f_kernel(const float* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx,
                                                                float* __restrict__ dx, PoolGeom g) {
  const int CV = g.C >> 2;
  const int total = g.N * g.H * g.W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int t = i / CV;
    const int ix = t % g.W;
    t /= g.W;
    const int iy = t % g.H, n = t / g.H;
    const int oy = iy / g.ph, ox = ix / g.pw;
    float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
    if (oy < g.OH && ox < g.OW) {
      const size_t o = ((size_t)(n * g.OH + oy) * g.OW + ox) * g.C + cv * 4;
      const int local = (iy - oy * g.ph) * g.pw + (ix - ox * g.pw);
      const float4 d = *reinterpret_cast<const float4*>(dy + o);
      const uint32_t ib = *reinterpret_cast<const uint32_t*>(idx + o);
      out.x = (int)(ib & 255) == local ? d.x : 0.f;
      out.y = (int)((ib >> 8) & 255) == local ? d.y : 0.f;
      out.z = (int)((ib >> 16) & 255) == local ? d.z : 0.f;
      out.w = (int)(ib >> 24) == local ? d.w : 0.f;
    }
    *reinterpret_cast<float4*>(dx + (size_t)i * 4) = out;
  }
}

// Overlapping windows (e.g. the ResNet-50 stem's 3x3 / stride 2 / pad 1), bf16, 8 channels per
// thread, 32-bit index math: the generic per-element kernels above are ALU bound on 64-bit div/mod
// chains (~0.4 ms per backward at 256 x 64 x 64 x 64). Forward: one 16-B load per in-image tap.
// Backward is a gather: each input vector visits the (<= ceil(ph/sh) x ceil(pw/sw)) windows that
// contain it and sums the gradients whose argmax is this position (the same sum the scalar kernel
// forms, in the same window order).
__global__ void __launch_bounds__(256) maxpool_fwd_ov8_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                              uint8_t* __restrict__ idx, PoolGeom g) {
  const int CV = g.C >> 3;
  const int total = g.N * g.OH * g.OW * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int t = i / CV;
    const int ox = t % g.OW;
    t /= g.OW;
    const int oy = t % g.OH, n = t / g.OH;
    float best[8], v[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int ky = 0; ky < g.ph; ++ky) {
      const int iy = oy * g.sh - g.padh + ky;
      if (iy < 0 || iy >= g.H) continue;
      for (int kx = 0; kx < g.pw; ++kx) {
        const int ix = ox * g.sw - g.padw + kx;
        if (ix < 0 || ix >= g.W) continue;
        unpack8(*reinterpret_cast<const uint4*>(x + ((size_t)(n * g.H + iy) * g.W + ix) * g.C + cv * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(ky * g.pw + kx); }
      }
    }
    *reinterpret_cast<uint4*>(y + (size_t)i * 8) = pack8(best);
    *reinterpret_cast<uint2*>(idx + (size_t)i * 8) = *reinterpret_cast<uint2*>(bi);
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_ov8_kernel(const bf16* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx, bf16* __restrict__ dx,
                                                              PoolGeom g) {
  const int CV = g.C >> 3;
  const int total = g.N * g.H * g.W * CV;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int t = i / CV;
    const int ix = t % g.W;
    t /= g.W;
    const int iy = t % g.H, n = t / g.H;
    const int oy0 = max(0, (iy + g.padh - g.ph + g.sh) / g.sh), oy1 = min(g.OH - 1, (iy + g.padh) / g.sh);
    const int ox0 = max(0, (ix + g.padw - g.pw + g.sw) / g.sw), ox1 = min(g.OW - 1, (ix + g.padw) / g.sw);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = iy - (oy * g.sh - g.padh);
      if (ky < 0 || ky >= g.ph) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = ix - (ox * g.sw - g.padw);
        if (kx < 0 || kx >= g.pw) continue;
        const size_t o = ((size_t)(n * g.OH + oy) * g.OW + ox) * g.C + cv * 8;
        const uint2 ib = *reinterpret_cast<const uint2*>(idx + o);
        const uint8_t* b = reinterpret_cast<const uint8_t*>(&ib);
        const int local = ky * g.pw + kx;
        float d[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), d);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (b[e] == local) acc[e] += d[e];
      }
    }
    *reinterpret_cast<uint4*>(dx + (size_t)i * 8) = pack8(acc);
  }
}

// The same gather fused with the backward statistics of the BatchNorm(+ReLU) whose output the
// pool consumed (the ResNet stem: conv -> BN -> ReLU -> maxpool). dy' = dy at the window's argmax
// where the pooled value (= that ReLU output) is > 0, else 0; per block (sum dy', sum dy' * xhat)
// rows go to slab[block][2][C] (xhat from the BN input x). Saves the full-resolution pass over dy
// and the ReLU output that a separate bn_partial would make. Requires C / 8 to divide 256 and the
// grid-stride to be a multiple of C / 8 (fixed channel group per thread).
__global__ void __launch_bounds__(256) maxpool_bwd_bnb_kernel(const bf16* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              const bf16* __restrict__ ypool,
                                                              const bf16* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ istd, bf16* __restrict__ dx,
                                                              PoolGeom g, float* __restrict__ slab,
                                                              float* __restrict__ zero_sums) {
  __shared__ float red[256 * 16];
  if (zero_sums && blockIdx.x == 0)  // the [2][C] sums bn_slab_reduce accumulates into
    for (int j = threadIdx.x; j < 2 * g.C; j += blockDim.x) zero_sums[j] = 0.f;
  const int CV = g.C / 8;
  const long total = (long)g.N * g.H * g.W * CV;
  const int cv = threadIdx.x % CV;  // fixed: blockDim and the grid stride are multiples of CV
  float mu[8], is[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cv * 8 + e];
    is[e] = istd[cv * 8 + e];
    s[e] = q[e] = 0.f;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i / CV;
    const int ix = (int)(t % g.W);
    t /= g.W;
    const int iy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    const int oy = iy / g.ph, ox = ix / g.pw;
    float out[8];
    if (oy < g.OH && ox < g.OW) {
      const long o = (((long)n * g.OH + oy) * g.OW + ox) * g.C + cv * 8;
      const int local = (iy - oy * g.ph) * g.pw + (ix - ox * g.pw);
      float d[8], yp[8], xv[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + o), d);
      unpack8(*reinterpret_cast<const uint4*>(ypool + o), yp);
      unpack8(*reinterpret_cast<const uint4*>(x + i * 8), xv);
      const uint2 ib = *reinterpret_cast<const uint2*>(idx + o);
      const uint8_t* b = reinterpret_cast<const uint8_t*>(&ib);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        out[e] = (b[e] == local && yp[e] > 0.f) ? d[e] : 0.f;
        s[e] += out[e];
        q[e] += out[e] * (xv[e] - mu[e]) * is[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = 0.f;
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8(out);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[threadIdx.x * 16 + e] = s[e];
    red[threadIdx.x * 16 + 8 + e] = q[e];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * g.C; j += blockDim.x) {
    const int which = j / g.C, c = j % g.C, grp = c / 8, e = c % 8;
    float a = 0.f;
    for (int tt = grp; tt < (int)blockDim.x; tt += CV) a += red[tt * 16 + which * 8 + e];
    slab[((long)blockIdx.x * 2 + which) * g.C + c] = a;
  }
}

template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, PoolGeom g) {
  const long total = (long)g.N * g.OH * g.OW * g.C;
  const float inv = 1.f / (float)(g.ph * g.pw);  // count_include_pad semantics (avgpool_ops.cu:53)
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    long t = i / g.C;
    const int ox = (int)(t % g.OW);
    t /= g.OW;
    const int oy = (int)(t % g.OH);
    const int n = (int)(t / g.OH);
    float s = 0.f;
    for (int ky = 0; ky < g.ph; ++ky) {
      const int iy = oy * g.sh - g.padh + ky;
      if (iy < 0 || iy >= g.H) continue;
      for (int kx = 0; kx < g.pw; ++kx) {
        const int ix = ox * g.sw - g.padw + kx;
        if (ix < 0 || ix >= g.W) continue;
        s += ld(x, (((long)n * g.H + iy) * g.W + ix) * g.C + c);
      }
    }
    y[i] = from_f<T>(s * inv);
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, PoolGeom g) {
  const long total = (long)g.N * g.H * g.W * g.C;
  const float inv = 1.f / (float)(g.ph * g.pw);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    long t = i / g.C;
    const int ix = (int)(t % g.W);
    t /= g.W;
    const int iy = (int)(t % g.H);
    const int n = (int)(t / g.H);
    const int oy0 = max(0, (iy + g.padh - g.ph + g.sh) / g.sh), oy1 = min(g.OH - 1, (iy + g.padh) / g.sh);
    const int ox0 = max(0, (ix + g.padw - g.pw + g.sw) / g.sw), ox1 = min(g.OW - 1, (ix + g.padw) / g.sw);
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int ky = iy - (oy * g.sh - g.padh);
      if (ky < 0 || ky >= g.ph) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kx = ix - (ox * g.sw - g.padw);
        if (kx < 0 || kx >= g.pw) continue;
        acc += ld(dy, (((long)n * g.OH + oy) * g.OW + ox) * g.C + c);
      }
    }
    dx[i] = from_f<T>(acc * inv);
  }
}

// Global average pool (window == whole image, stride irrelevant): one wave per (n, 64 channels)
template <typename T>
__global__ void global_avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int HW, int C) {
  const long total = (long)N * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int n = (int)(i / C);
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += ld(x, ((long)n * HW + p) * C + c);
    y[i] = from_f<T>(s / (float)HW);
  }
}

template <typename T>
__global__ void global_avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  const long total = (long)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((long)HW * C));
    dx[i] = from_f<T>(ld(dy, (long)n * C + c) * inv);
  }
}

// ----------------------------------- activations -----------------------------------------
enum Act { kRelu = 0, kLeaky = 1, kElu = 2, kSigmoid = 3, kTanh = 4, kLinear = 5 };

__device__ __forceinline__ float act_f(int t, float x, float a) {
  switch (t) {
    case kRelu: return fmaxf(x, 0.f);
    case kLeaky: return x > 0.f ? x : a * x;
    case kElu: return x > 0.f ? x : a * (__expf(x) - 1.f);
    case kSigmoid: return 1.f / (1.f + __expf(-x));
    case kTanh: return tanhf(x);
    default: return x;
  }
}
__device__ __forceinline__ float act_df(int t, float x, float a) {
  switch (t) {
    case kRelu: return x > 0.f ? 1.f : 0.f;
    case kLeaky: return x > 0.f ? 1.f : a;
    case kElu: return x > 0.f ? 1.f : a * __expf(x);
    case kSigmoid: { const float s = 1.f / (1.f + __expf(-x)); return s * (1.f - s); }
    case kTanh: { const float t2 = tanhf(x); return 1.f - t2 * t2; }
    default: return 1.f;
  }
}

template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long n, int type, float alpha) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float f[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) f[v] = act_f(type, ld(x, i * 8 + v), alpha);
#pragma unroll
    for (int v = 0; v < 8; ++v) y[i * 8 + v] = from_f<T>(f[v]);
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = from_f<T>(act_f(type, ld(x, i), alpha));
}

template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx, long n, int type,
                               float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = from_f<T>(ld(dy, i) * act_df(type, ld(x, i), alpha));
}

// softmax over the innermost dim (channels in NHWC): one wave per row
template <typename T>
__global__ void softmax_rows_kernel(const T* __restrict__ x, T* __restrict__ y, long rows, int C) {
  const int lane = threadIdx.x & 63;
  const long row = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  if (row >= rows) return;
  const T* xr = x + row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, ld(xr, c));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(ld(xr, c) - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int c = lane; c < C; c += 64) y[row * C + c] = from_f<T>(__expf(ld(xr, c) - m) * inv);
}

template <typename T>
__global__ void softmax_rows_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy, T* __restrict__ dx,
                                        long rows, int C) {
  const int lane = threadIdx.x & 63;
  const long row = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  if (row >= rows) return;
  float d = 0.f;
  for (int c = lane; c < C; c += 64) d += ld(y, row * C + c) * ld(dy, row * C + c);
  d = wave_sum(d);
  for (int c = lane; c < C; c += 64) {
    const long o = row * C + c;
    dx[o] = from_f<T>(ld(y, o) * (ld(dy, o) - d));
  }
}

// ------------------------------------- dropout -------------------------------------------
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, float p, uint64_t seed,
                               const uint64_t* __restrict__ ctr) {
  const float scale = 1.f / (1.f - p);
  // device-side draw counter: a hipGraph replay captures `seed` as a constant, the counter slot is
  // rewritten by counter_bump before every replayed forward, so each replay draws a new mask
  if (ctr) seed += ctr[0] * 0x9E3779B97F4A7C15ull;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n + 3) / 4; i += (long)gridDim.x * blockDim.x) {
    const uint4 r = Philox::gen(seed, (uint64_t)i);
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const long o = i * 4 + v;
      if (o < n) y[o] = from_f<T>(Philox::u01(rr[v]) >= p ? ld(x, o) * scale : 0.f);
    }
  }
}

// slot = ++ctr (one thread): per-forward draw index for dropout, advanced inside the graph
__global__ void counter_bump_kernel(uint64_t* ctr, uint64_t* slot) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const uint64_t v = ctr[0] + 1;
    ctr[0] = v;
    slot[0] = v;
  }
}

// -------------------------------- layout / conversion ------------------------------------
// x NCHW (float) -> y NHWC (T)
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int HW) {
  const long total = (long)N * C * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long t = i / C;
    const int p = (int)(t % HW);
    const int n = (int)(t / HW);
    y[i] = from_f<T>(x[((long)n * C + c) * HW + p]);
  }
}

// x NCHW (float, C channels) -> y NHWC (T, Cp >= C channels, zero padded)
template <typename T>
__global__ void nchw_to_nhwc_pad_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int Cp, int HW) {
  const long total = (long)N * Cp * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long t = i / Cp;
    const int p = (int)(t % HW);
    const int n = (int)(t / HW);
    y[i] = from_f<T>(c < C ? x[((long)n * C + c) * HW + p] : 0.f);
  }
}

// W[co][t][ci] -> Wt[ci][t][co]   (dgrad operand), source fp32 or bf16, dest bf16
template <typename S>
__global__ void conv_weight_transpose_kernel(const S* __restrict__ w, bf16* __restrict__ wt, int Co, int T_, int Ci) {
  const long total = (long)Co * T_ * Ci;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    // i indexes the destination
    const int co = (int)(i % Co);
    long r = i / Co;
    const int t = (int)(r % T_);
    const int ci = (int)(r / T_);
    wt[i] = (bf16)to_f(w[((long)co * T_ + t) * Ci + ci]);
  }
}

// All dgrad weight operands of a model in ONE launch: table rows are
// {src ptr, dst ptr, Co, taps, Ci}; blockIdx.y selects the tensor.
// [Co][T][Ci] -> [Ci][T][Co] for every conv of a model in one launch (blockIdx.y = conv). Each
// workgroup moves one 64(co) x 64(ci) tile of one tap through LDS: 16-byte coalesced loads along
// ci, 16-byte coalesced stores along co (Ci, Co multiples of 8, 256-byte aligned arena views).
// T = bf16 (the bf16 compute path's operands) or float (the exact fp32 path's): 16-byte vectors of
// V = 16 / sizeof(T) elements; Ci, Co multiples of V.
template <typename T>
__global__ void __launch_bounds__(256) multi_weight_transpose_kernel(const int64_t* __restrict__ table) {
  constexpr int V = 16 / (int)sizeof(T), RV = 64 / V;  // elements per vector, vectors per 64-row
  const int64_t* e = table + blockIdx.y * 5;
  const T* w = reinterpret_cast<const T*>(e[0]);
  T* wt = reinterpret_cast<T*>(e[1]);
  const int Co = (int)e[2], T_ = (int)e[3], Ci = (int)e[4];
  const int tco = (Co + 63) / 64, tci = (Ci + 63) / 64;
  int b = blockIdx.x;
  if (b >= T_ * tco * tci) return;  // this conv has fewer tiles than the largest one
  const int t = b % T_;
  b /= T_;
  const int ic = b % tci, oc = b / tci;
  __shared__ T tile[64][64 + V];  // row pitch keeps the 16-byte row chunks aligned
  for (int k = threadIdx.x; k < 64 * RV; k += 256) {
    const int r = k / RV, cv = (k % RV) * V;
    const int co = oc * 64 + r, ci = ic * 64 + cv;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (co < Co && ci < Ci) v = *reinterpret_cast<const uint4*>(w + ((long)co * T_ + t) * Ci + ci);
    *reinterpret_cast<uint4*>(&tile[r][cv]) = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * RV; k += 256) {
    const int r = k / RV, cv = (k % RV) * V;  // r: ci within the tile, cv: first of V co
    const int ci = ic * 64 + r, co = oc * 64 + cv;
    if (ci < Ci && co < Co) {
      uint4 v;
      T* o = reinterpret_cast<T*>(&v);
#pragma unroll
      for (int j = 0; j < V; ++j) o[j] = tile[cv + j][r];
      *reinterpret_cast<uint4*>(wt + ((long)ci * T_ + t) * Co + co) = v;
    }
  }
}

void multi_weight_transpose(const int64_t* table, int n, long max_tiles, hipStream_t s, int f32) {
  if (n <= 0) return;
  if (f32)
    hipLaunchKernelGGL(multi_weight_transpose_kernel<float>, dim3((unsigned)max_tiles, n), dim3(256), 0, s, table);
  else
    hipLaunchKernelGGL(multi_weight_transpose_kernel<bf16>, dim3((unsigned)max_tiles, n), dim3(256), 0, s, table);
  DCNN_LAUNCH_CHECK();
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (bf16)x[i];
}

// ------------------------------ im2col / col2im (NCHW, fp32) -----------------------------
// col[(c,kh,kw)][n*OH*OW + oh*OW + ow]   (the reference's column layout, tensor_kernels.cu:18)
__global__ void im2col_kernel(const float* __restrict__ x, float* __restrict__ col, int N, int C, int H, int W,
                              int KH, int KW, int SH, int SW, int PH, int PW, int OH, int OW) {
  const long cols = (long)N * OH * OW;
  const long total = (long)C * KH * KW * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long j = i % cols;
    const int r = (int)(i / cols);
    const int kw = r % KW, kh = (r / KW) % KH, c = r / (KW * KH);
    const int ow = (int)(j % OW), oh = (int)((j / OW) % OH), n = (int)(j / ((long)OW * OH));
    const int iy = oh * SH - PH + kh, ix = ow * SW - PW + kw;
    col[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? x[(((long)n * C + c) * H + iy) * W + ix] : 0.f;
  }
}

__global__ void col2im_kernel(const float* __restrict__ col, float* __restrict__ x, int N, int C, int H, int W,
                              int KH, int KW, int SH, int SW, int PH, int PW, int OH, int OW) {
  const long total = (long)N * C * H * W;
  const long cols = (long)N * OH * OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ix = (int)(i % W), iy = (int)((i / W) % H), c = (int)((i / ((long)W * H)) % C);
    const int n = (int)(i / ((long)W * H * C));
    float acc = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int ty = iy + PH - kh;
      if (ty < 0 || ty % SH) continue;
      const int oh = ty / SH;
      if (oh >= OH) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tx = ix + PW - kw;
        if (tx < 0 || tx % SW) continue;
        const int ow = tx / SW;
        if (ow >= OW) continue;
        acc += col[((long)(c * KH + kh) * KW + kw) * cols + ((long)n * OH + oh) * OW + ow];
      }
    }
    x[i] = acc;
  }
}

// ------------------------------------- launchers -----------------------------------------
#define DCNN_DT(dtype, FN, ...) \
  if (dtype == 0) FN<float>(__VA_ARGS__); else FN<bf16>(__VA_ARGS__)

static bool pool_nov8(const PoolGeom& g) {
  return g.C % 8 == 0 && g.sh == g.ph && g.sw == g.pw && g.padh == 0 && g.padw == 0;
}
// fp32 non-overlapping windows: 4-channel vectors, 32-bit indices
static bool pool_nov4f(const PoolGeom& g) {
  return g.C % 4 == 0 && g.sh == g.ph && g.sw == g.pw && g.padh == 0 && g.padw == 0 && g.ph * g.pw <= 255 &&
         (long)g.N * g.H * g.W * g.C < (1L << 31);
}
// vectorised overlapping-window kernels: 8-channel vectors, 32-bit indices, windows of <= 255 taps
static bool pool_ov8(const PoolGeom& g) {
  return g.C % 8 == 0 && g.ph * g.pw <= 255 && (long)g.N * g.H * g.W * g.C < (1L << 31);
}

template <typename T>
static void maxpool_fwd_t(const void* x, void* y, uint8_t* idx, PoolGeom g, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {
    if (pool_nov4f(g)) {
      const long total = (long)g.N * g.OH * g.OW * g.C / 4;
      hipLaunchKernelGGL(maxpool_fwd_nov4f_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const float*)x,
                         (float*)y, idx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pool_nov8(g)) {
      const long total = (long)g.N * g.OH * g.OW * g.C / 8;
      hipLaunchKernelGGL(maxpool_fwd_nov8_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)x, (bf16*)y,
                         idx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pool_ov8(g)) {
      const long total = (long)g.N * g.OH * g.OW * g.C / 8;
      hipLaunchKernelGGL(maxpool_fwd_ov8_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)x, (bf16*)y,
                         idx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  const long total = (long)g.N * g.OH * g.OW * g.C;
  hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)x, (T*)y, idx, g);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void maxpool_bwd_t(const void* dy, const uint8_t* idx, void* dx, PoolGeom g, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {
    if (pool_nov4f(g)) {
      const long total = (long)g.N * g.H * g.W * g.C / 4;
      hipLaunchKernelGGL(maxpool_bwd_nov4f_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const float*)dy, idx,
                         (float*)dx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pool_nov8(g)) {
      const long total = (long)g.N * g.H * g.W * g.C / 8;
      hipLaunchKernelGGL(maxpool_bwd_nov8_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)dy, idx,
                         (bf16*)dx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pool_ov8(g)) {
      const long total = (long)g.N * g.H * g.W * g.C / 8;
      hipLaunchKernelGGL(maxpool_bwd_ov8_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)dy, idx,
                         (bf16*)dx, g);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  const long total = (long)g.N * g.H * g.W * g.C;
  hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)dy, idx, (T*)dx, g);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void avgpool_fwd_t(const void* x, void* y, PoolGeom g, hipStream_t s) {
  if (g.OH == 1 && g.OW == 1 && g.ph == g.H && g.pw == g.W && g.padh == 0 && g.padw == 0) {
    const long total = (long)g.N * g.C;
    hipLaunchKernelGGL(global_avgpool_fwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)x, (T*)y,
                       g.N, g.H * g.W, g.C);
  } else {
    const long total = (long)g.N * g.OH * g.OW * g.C;
    hipLaunchKernelGGL(avgpool_fwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)x, (T*)y, g);
  }
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void avgpool_bwd_t(const void* dy, void* dx, PoolGeom g, hipStream_t s) {
  const long total = (long)g.N * g.H * g.W * g.C;
  if (g.OH == 1 && g.OW == 1 && g.ph == g.H && g.pw == g.W && g.padh == 0 && g.padw == 0)
    hipLaunchKernelGGL(global_avgpool_bwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)dy, (T*)dx,
                       g.N, g.H * g.W, g.C);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const T*)dy, (T*)dx, g);
  DCNN_LAUNCH_CHECK();
}

// Same result per element as maxpool_bwd_bnb_kernel for windows that tile the input exactly
// (H % ph == 0, W % pw == 0): one thread per POOLED vector walks its window, so the pooled
// gradient / pooled output / argmax are read once instead of once per window pixel and the
// index arithmetic is 32-bit and per window (the per-pixel 64-bit div/mod chains of the generic
// kernel made it ALU bound). Statistics partials per block in the same [blocks][2][C] layout.
// (P > 0: a compile-time P x P window, its x loads issued together)
template <int P>
__global__ void __launch_bounds__(256) maxpool_bwd_bnb_w_kernel(const bf16* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx,
                                                                const bf16* __restrict__ ypool,
                                                                const bf16* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ istd,
                                                                bf16* __restrict__ dx, PoolGeom g,
                                                                float* __restrict__ slab,
                                                                float* __restrict__ zero_sums) {
  __shared__ float red[256 * 16];
  if (zero_sums && blockIdx.x == 0)
    for (int j = threadIdx.x; j < 2 * g.C; j += blockDim.x) zero_sums[j] = 0.f;
  const unsigned CV = g.C / 8;
  const unsigned total = (unsigned)g.N * g.OH * g.OW * CV;
  const int cv = threadIdx.x % CV;  // fixed: blockDim and the grid stride are multiples of CV
  float mu[8], is[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cv * 8 + e];
    is[e] = istd[cv * 8 + e];
    s[e] = q[e] = 0.f;
  }
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    unsigned t = i / CV;
    const int ox = (int)(t % g.OW);
    t /= g.OW;
    const int oy = (int)(t % g.OH);
    const int n = (int)(t / g.OH);
    float d[8], yp[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + (size_t)i * 8), d);
    unpack8(*reinterpret_cast<const uint4*>(ypool + (size_t)i * 8), yp);
    const uint2 ib = *reinterpret_cast<const uint2*>(idx + (size_t)i * 8);
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&ib);
    auto put = [&](const uint4& raw, int local, size_t xi) {
      float xv[8], out[8];
      unpack8(raw, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        out[e] = (b[e] == local && yp[e] > 0.f) ? d[e] : 0.f;
        s[e] += out[e];
        q[e] += out[e] * (xv[e] - mu[e]) * is[e];
      }
      *reinterpret_cast<uint4*>(dx + xi) = pack8(out);
    };
    if constexpr (P > 0) {
      size_t xi[P * P];
      uint4 w[P * P];
#pragma unroll
      for (int ky = 0; ky < P; ++ky)
#pragma unroll
        for (int kx = 0; kx < P; ++kx) {
          xi[ky * P + kx] = (((size_t)n * g.H + oy * P + ky) * g.W + ox * P + kx) * g.C + cv * 8;
          w[ky * P + kx] = *reinterpret_cast<const uint4*>(x + xi[ky * P + kx]);
        }
#pragma unroll
      for (int k = 0; k < P * P; ++k) put(w[k], k, xi[k]);
    } else {
      for (int ky = 0; ky < g.ph; ++ky)
        for (int kx = 0; kx < g.pw; ++kx) {
          const size_t xi = (((size_t)n * g.H + oy * g.ph + ky) * g.W + ox * g.pw + kx) * g.C + cv * 8;
          put(*reinterpret_cast<const uint4*>(x + xi), ky * g.pw + kx, xi);
        }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[threadIdx.x * 16 + e] = s[e];
    red[threadIdx.x * 16 + 8 + e] = q[e];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * g.C; j += blockDim.x) {
    const int which = j / g.C, c = j % g.C, grp = c / 8, e = c % 8;
    float a = 0.f;
    for (int tt = grp; tt < (int)blockDim.x; tt += CV) a += red[tt * 16 + which * 8 + e];
    slab[((long)blockIdx.x * 2 + which) * g.C + c] = a;
  }
}

static int bnb_pool_blocks(const PoolGeom& g) {
  const long total = (long)g.N * g.H * g.W * g.C / 8;
  return grid_for(total, 256, 1024);
}

bool maxpool_bwd_bnb_supported(PoolGeom g) { return pool_nov8(g) && 256 % (g.C / 8) == 0; }

int maxpool_bwd_bnb_rows(PoolGeom g) { return bnb_pool_blocks(g); }

void maxpool_bwd_bnb(const bf16* dy, const uint8_t* idx, const bf16* ypool, const bf16* x, const float* mean,
                     const float* istd, bf16* dx, PoolGeom g, float* slab, float* zero_sums, hipStream_t s) {
  if (!maxpool_bwd_bnb_supported(g)) throw std::runtime_error("maxpool_bwd_bnb: unsupported geometry");
  if (g.H % g.ph == 0 && g.W % g.pw == 0 && g.OH == g.H / g.ph && g.OW == g.W / g.pw &&
      (long)g.N * g.H * g.W * g.C < (1l << 31)) {
    hipLaunchKernelGGL((g.ph == 2 && g.pw == 2) ? maxpool_bwd_bnb_w_kernel<2> : maxpool_bwd_bnb_w_kernel<0>,
                       dim3(bnb_pool_blocks(g)), dim3(256), 0, s, dy, idx, ypool, x, mean,
                       istd, dx, g, slab, zero_sums);
    DCNN_LAUNCH_CHECK();
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_bnb_kernel, dim3(bnb_pool_blocks(g)), dim3(256), 0, s, dy, idx, ypool, x, mean, istd,
                     dx, g, slab, zero_sums);
  DCNN_LAUNCH_CHECK();
}

void maxpool_fwd(int dt, const void* x, void* y, uint8_t* idx, PoolGeom g, hipStream_t s) { DCNN_DT(dt, maxpool_fwd_t, x, y, idx, g, s); }
void maxpool_bwd(int dt, const void* dy, const uint8_t* idx, void* dx, PoolGeom g, hipStream_t s) { DCNN_DT(dt, maxpool_bwd_t, dy, idx, dx, g, s); }
void avgpool_fwd(int dt, const void* x, void* y, PoolGeom g, hipStream_t s) { DCNN_DT(dt, avgpool_fwd_t, x, y, g, s); }
void avgpool_bwd(int dt, const void* dy, void* dx, PoolGeom g, hipStream_t s) { DCNN_DT(dt, avgpool_bwd_t, dy, dx, g, s); }

template <typename T>
static void act_fwd_t(const void* x, void* y, long n, int type, float a, hipStream_t s) {
  hipLaunchKernelGGL(act_fwd_kernel<T>, dim3(grid_for(n / 8 + 1, 256)), dim3(256), 0, s, (const T*)x, (T*)y, n, type, a);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void act_bwd_t(const void* x, const void* dy, void* dx, long n, int type, float a, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(grid_for(n, 256)), dim3(256), 0, s, (const T*)x, (const T*)dy, (T*)dx, n,
                     type, a);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void softmax_t(const void* x, void* y, long rows, int C, hipStream_t s) {
  hipLaunchKernelGGL(softmax_rows_kernel<T>, dim3((rows * 64 + 255) / 256), dim3(256), 0, s, (const T*)x, (T*)y, rows, C);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void softmax_bwd_t(const void* y, const void* dy, void* dx, long rows, int C, hipStream_t s) {
  hipLaunchKernelGGL(softmax_rows_bwd_kernel<T>, dim3((rows * 64 + 255) / 256), dim3(256), 0, s, (const T*)y,
                     (const T*)dy, (T*)dx, rows, C);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void dropout_t(const void* x, void* y, long n, float p, uint64_t seed, const uint64_t* ctr, hipStream_t s) {
  hipLaunchKernelGGL(dropout_kernel<T>, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, s, (const T*)x, (T*)y, n, p, seed,
                     ctr);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void nchw_to_nhwc_t(const float* x, void* y, int N, int C, int HW, hipStream_t s) {
  hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(grid_for((long)N * C * HW, 256)), dim3(256), 0, s, x, (T*)y, N, C, HW);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void nchw_to_nhwc_pad_t(const float* x, void* y, int N, int C, int Cp, int HW, hipStream_t s) {
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel<T>, dim3(grid_for((long)N * Cp * HW, 256)), dim3(256), 0, s, x, (T*)y, N, C,
                     Cp, HW);
  DCNN_LAUNCH_CHECK();
}
template <typename T>
static void wt_t(const void* w, bf16* wt, int Co, int T_, int Ci, hipStream_t s) {
  hipLaunchKernelGGL(conv_weight_transpose_kernel<T>, dim3(grid_for((long)Co * T_ * Ci, 256)), dim3(256), 0, s,
                     (const T*)w, wt, Co, T_, Ci);
  DCNN_LAUNCH_CHECK();
}

void act_fwd(int dt, const void* x, void* y, long n, int type, float a, hipStream_t s) { DCNN_DT(dt, act_fwd_t, x, y, n, type, a, s); }
void act_bwd(int dt, const void* x, const void* dy, void* dx, long n, int type, float a, hipStream_t s) { DCNN_DT(dt, act_bwd_t, x, dy, dx, n, type, a, s); }
void softmax_rows(int dt, const void* x, void* y, long rows, int C, hipStream_t s) { DCNN_DT(dt, softmax_t, x, y, rows, C, s); }
void softmax_rows_bwd(int dt, const void* y, const void* dy, void* dx, long rows, int C, hipStream_t s) { DCNN_DT(dt, softmax_bwd_t, y, dy, dx, rows, C, s); }
void dropout(int dt, const void* x, void* y, long n, float p, uint64_t seed, const uint64_t* ctr, hipStream_t s) {
  DCNN_DT(dt, dropout_t, x, y, n, p, seed, ctr, s);
}
void counter_bump(uint64_t* ctr, uint64_t* slot, hipStream_t s) {
  hipLaunchKernelGGL(counter_bump_kernel, dim3(1), dim3(64), 0, s, ctr, slot);
  DCNN_LAUNCH_CHECK();
}
void nchw_to_nhwc(int dt, const float* x, void* y, int N, int C, int HW, hipStream_t s) { DCNN_DT(dt, nchw_to_nhwc_t, x, y, N, C, HW, s); }
void nchw_to_nhwc_pad(int dt, const float* x, void* y, int N, int C, int Cp, int HW, hipStream_t s) { DCNN_DT(dt, nchw_to_nhwc_pad_t, x, y, N, C, Cp, HW, s); }
void conv_weight_transpose(int src_dt, const void* w, bf16* wt, int Co, int T_, int Ci, hipStream_t s) { DCNN_DT(src_dt, wt_t, w, wt, Co, T_, Ci, s); }
void cast_f32_bf16(const float* x, bf16* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, y, n);
  DCNN_LAUNCH_CHECK();
}
void im2col(const float* x, float* col, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW,
            int OH, int OW, hipStream_t s) {
  const long total = (long)C * KH * KW * N * OH * OW;
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, x, col, N, C, H, W, KH, KW, SH, SW, PH,
                     PW, OH, OW);
  DCNN_LAUNCH_CHECK();
}
void col2im(const float* col, float* x, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW,
            int OH, int OW, hipStream_t s) {
  const long total = (long)N * C * H * W;
  hipLaunchKernelGGL(col2im_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, col, x, N, C, H, W, KH, KW, SH, SW, PH,
                     PW, OH, OW);
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
