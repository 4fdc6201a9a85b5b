// Explicit im2col + GEMM convolution path (NHWC, bf16 or fp32), the second conv algorithm next
// to the implicit-GEMM / halo kernels. The reference lowers every conv this way (im2col into a
// column buffer, then one cuBLAS GEMM; src/nn/layers_impl/cuda/conv2d_ops.cu:78-98 and the
// column kernels of src/tensor/cuda/tensor_kernels.cu:18-135). Here the column matrix is the
// K-contiguous A operand of the bf16 MFMA GEMM (gemm2.hip, PLAIN mode), so the GEMM is a plain
// read-once NT GEMM with the usual fused epilogue; the price is materialising M x (KH*KW*C)
// elements in HBM. Used where it is asked for (DCNN_CONV_ALGO=im2col / set_conv_algo) and as an
// independent cross-check of the implicit kernels in the tests.
//
//   im2col:  col[m][(ky*KW + kx)*C + c] = x[n][oy*SH - PH + ky][ox*SW - PW + kx][c]  (0 outside)
//   col2im:  x[n][iy][ix][c] (+)= sum over (ky, kx) reaching it of col[m(ky,kx)][k(ky,kx,c)]
//            with the column index either tap-major (ky,kx,c) or channel-major (c,ky,kx): the
//            dgrad GEMM against the transposed weight [C][KH][KW][Co] produces channel-major rows.
// col2im is a gather (each input element sums its own taps in a fixed order): no atomics, so the
// result is deterministic. 16-byte vectors of 8 channels (C % 8 == 0).
#include "common.h"
#include "api.h"

namespace dcnn {

namespace {
template <typename T>
struct Vec8;
template <>
struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }
  static __device__ __forceinline__ void store(bf16* p, const float* f) { *reinterpret_cast<uint4*>(p) = pack8(f); }
  static __device__ __forceinline__ void copy(const bf16* s, bf16* d) {
    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
  }
  static __device__ __forceinline__ void zero(bf16* d) { *reinterpret_cast<uint4*>(d) = make_uint4(0, 0, 0, 0); }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* f) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
  static __device__ __forceinline__ void copy(const float* s, float* d) {
    *reinterpret_cast<float4*>(d) = *reinterpret_cast<const float4*>(s);
    *reinterpret_cast<float4*>(d + 4) = *reinterpret_cast<const float4*>(s + 4);
  }
  static __device__ __forceinline__ void zero(float* d) {
    *reinterpret_cast<float4*>(d) = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(d + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
};
}  // namespace

// one thread per (output pixel m, tap, 8-channel group): consecutive threads walk the channel
// groups of one tap, so both the gather read and the column write are contiguous 16-byte runs
template <typename T>
__global__ void im2col_nhwc_kernel(const T* __restrict__ x, T* __restrict__ col, ConvGeom g) {
  const int CG = g.C / 8, taps = g.KH * g.KW;
  const long total = (long)g.N * g.OH * g.OW * taps * CG;
  const long K = (long)taps * g.C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long r = i / CG;
    const int t = (int)(r % taps);
    const long m = r / taps;
    const int ox = (int)(m % g.OW), oy = (int)((m / g.OW) % g.OH), n = (int)(m / ((long)g.OW * g.OH));
    const int ky = t / g.KW, kx = t % g.KW;
    const int iy = oy * g.SH - g.PH + ky, ix = ox * g.SW - g.PW + kx;
    T* dst = col + m * K + (long)t * g.C + cg * 8;
    if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
      Vec8<T>::copy(x + (((long)n * g.H + iy) * g.W + ix) * g.C + cg * 8, dst);
    else
      Vec8<T>::zero(dst);
  }
}

// one thread per (input pixel, 8-channel group); taps summed in (ky, kx) order
template <typename T>
__global__ void col2im_nhwc_kernel(const T* __restrict__ col, T* __restrict__ x, const T* __restrict__ residual,
                                   ConvGeom g, int chan_major) {
  const int CG = g.C / 8, taps = g.KH * g.KW;
  const long total = (long)g.N * g.H * g.W * CG;
  const long K = (long)taps * g.C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long pix = i / CG;
    const int ix = (int)(pix % g.W), iy = (int)((pix / g.W) % g.H), n = (int)(pix / ((long)g.W * g.H));
    float acc[8];
    if (residual) {
      Vec8<T>::load(residual + pix * g.C + cg * 8, acc);
    } else {
#pragma unroll
      for (int v = 0; v < 8; ++v) acc[v] = 0.f;
    }
    for (int ky = 0; ky < g.KH; ++ky) {
      const int ty = iy + g.PH - ky;
      if (ty < 0 || ty % g.SH) continue;
      const int oy = ty / g.SH;
      if (oy >= g.OH) continue;
      for (int kx = 0; kx < g.KW; ++kx) {
        const int tx = ix + g.PW - kx;
        if (tx < 0 || tx % g.SW) continue;
        const int ox = tx / g.SW;
        if (ox >= g.OW) continue;
        const long m = ((long)n * g.OH + oy) * g.OW + ox;
        const int t = ky * g.KW + kx;
        float v8[8];
        if (!chan_major) {
          Vec8<T>::load(col + m * K + (long)t * g.C + cg * 8, v8);
        } else {
          const T* src = col + m * K + (long)(cg * 8) * taps + t;
#pragma unroll
          for (int v = 0; v < 8; ++v) v8[v] = (float)src[v * taps];
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) acc[v] += v8[v];
      }
    }
    Vec8<T>::store(x + pix * g.C + cg * 8, acc);
  }
}

static void check_geom(const ConvGeom& g) {
  if (g.C % 8 || g.N <= 0 || g.KH <= 0 || g.KW <= 0 || g.SH <= 0 || g.SW <= 0 || g.OH <= 0 || g.OW <= 0)
    throw std::runtime_error("im2col_nhwc: need C % 8 == 0 and a valid geometry");
  if ((g.H + 2 * g.PH - g.KH) / g.SH + 1 != g.OH || (g.W + 2 * g.PW - g.KW) / g.SW + 1 != g.OW)
    throw std::runtime_error("im2col_nhwc: output size does not match the geometry");
}

void im2col_nhwc(int dt, const void* x, void* col, const ConvGeom& g, hipStream_t s) {
  check_geom(g);
  const long total = (long)g.N * g.OH * g.OW * g.KH * g.KW * (g.C / 8);
  if (dt == 1)
    hipLaunchKernelGGL(im2col_nhwc_kernel<bf16>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)x, (bf16*)col, g);
  else
    hipLaunchKernelGGL(im2col_nhwc_kernel<float>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const float*)x, (float*)col, g);
  DCNN_LAUNCH_CHECK();
}

void col2im_nhwc(int dt, const void* col, void* x, const void* residual, const ConvGeom& g, int chan_major,
                 hipStream_t s) {
  check_geom(g);
  const long total = (long)g.N * g.H * g.W * (g.C / 8);
  if (dt == 1)
    hipLaunchKernelGGL(col2im_nhwc_kernel<bf16>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const bf16*)col,
                       (bf16*)x, (const bf16*)residual, g, chan_major);
  else
    hipLaunchKernelGGL(col2im_nhwc_kernel<float>, dim3(grid_for(total, 256)), dim3(256), 0, s, (const float*)col,
                       (float*)x, (const float*)residual, g, chan_major);
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
