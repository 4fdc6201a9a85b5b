// Gradient wire-format kernels for the data-parallel bf16 all-reduce (parallel/dp.py).
//
// On the GPU a bucket is packed to bf16 (grad_pack), reduce-scattered and all-gathered by RCCL
// in bf16 (collectives only: they capture into the step's hipGraph), and expanded back into the
// fp32 gradient arena (grad_unpack): half the wire bytes of the fp32 all-reduce. grad_sum_chunks
// is the fixed rank-order fp32 sum of w bf16 shard copies (one rounding), the reduction of the
// all_to_all form of the same wire format. All passes are HBM-bound streams: 16-byte vector
// loads/stores, grid-stride.
#include "api.h"
#include "common.h"

namespace dcnn {

namespace {

// 8 fp32 -> 8 bf16 (x scale)
__global__ void grad_pack_kernel(const float* __restrict__ g, bf16* __restrict__ out, long n, float scale) {
  const long n8 = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(g + i * 8);
    const f32x4 b = *reinterpret_cast<const f32x4*>(g + i * 8 + 4);
    bf16x8 o;
    for (int k = 0; k < 4; ++k) {
      o[k] = (bf16)(a[k] * scale);
      o[k + 4] = (bf16)(b[k] * scale);
    }
    *reinterpret_cast<bf16x8*>(out + i * 8) = o;
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (bf16)(g[i] * scale);
}

// dst[i] = bf16( sum_{r=0..w-1} src[r*ld + i] )   (fp32 accumulation in rank order)
__global__ void grad_sum_chunks_kernel(const bf16* __restrict__ src, int w, long ld, long n, bf16* __restrict__ dst) {
  const long n8 = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    float acc[8];
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int r = 0; r < w; ++r) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + r * ld + i * 8);
      for (int k = 0; k < 8; ++k) acc[k] += (float)v[k];
    }
    bf16x8 o;
    for (int k = 0; k < 8; ++k) o[k] = (bf16)acc[k];
    *reinterpret_cast<bf16x8*>(dst + i * 8) = o;
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int r = 0; r < w; ++r) acc += (float)src[r * ld + i];
    dst[i] = (bf16)acc;
  }
}

__global__ void grad_unpack_kernel(const bf16* __restrict__ in, float* __restrict__ g, long n) {
  const long n8 = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + i * 8);
    f32x4 a, b;
    for (int k = 0; k < 4; ++k) {
      a[k] = (float)v[k];
      b[k] = (float)v[k + 4];
    }
    *reinterpret_cast<f32x4*>(g + i * 8) = a;
    *reinterpret_cast<f32x4*>(g + i * 8 + 4) = b;
  }
  for (long i = n8 * 8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) g[i] = (float)in[i];
}

inline int stream_grid(long n) { return grid_for((n + 7) / 8, 256); }

}  // namespace

// byte-exact zero fill (16-byte stores + tail). Used instead of hipMemsetAsync for buffers zeroed
// inside captured graphs: on ROCm 7.2 a captured memset node wrote garbage from its second replay
// on (tools/dbg/memset_graph.py), a kernel node replays correctly.
__global__ void zero_bytes_kernel(unsigned char* __restrict__ p, long nbytes) {
  const long n16 = nbytes / 16;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (long i = n16 * 16 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < nbytes; i += stride) p[i] = 0;
}

void zero_bytes(void* p, long nbytes, hipStream_t s) {
  if (nbytes <= 0) return;
  if (reinterpret_cast<uintptr_t>(p) % 16) throw std::runtime_error("zero_bytes: 16-byte aligned buffers only");
  hipLaunchKernelGGL(zero_bytes_kernel, dim3(grid_for((nbytes + 15) / 16, 256)), dim3(256), 0, s,
                     static_cast<unsigned char*>(p), nbytes);
  DCNN_LAUNCH_CHECK();
}

// two device-to-device copies in one launch (a training step's batch and labels into the captured
// graph's static slots: the runtime's blit kernel took ~7 + ~5 us for 12.6 MB + 2 KB). 16-byte
// moves where both pointers are 16-byte aligned, bytes otherwise; blockIdx.y picks the pair.
__global__ void copy_pair_kernel(unsigned char* __restrict__ d0, const unsigned char* __restrict__ s0, long n0,
                                 unsigned char* __restrict__ d1, const unsigned char* __restrict__ s1, long n1) {
  unsigned char* d = blockIdx.y ? d1 : d0;
  const unsigned char* s = blockIdx.y ? s1 : s0;
  const long n = blockIdx.y ? n1 : n0;
  const long stride = (long)gridDim.x * blockDim.x;
  const bool vec = ((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15) == 0;
  const long n16 = vec ? n / 16 : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
  for (long i = n16 * 16 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

void copy_pair(void* d0, const void* s0, long n0, void* d1, const void* s1, long n1, hipStream_t s) {
  const long m = n0 > n1 ? n0 : n1;
  if (m <= 0) return;
  hipLaunchKernelGGL(copy_pair_kernel, dim3(grid_for((m + 15) / 16, 256), 2), dim3(256), 0, s,
                     static_cast<unsigned char*>(d0), static_cast<const unsigned char*>(s0), n0,
                     static_cast<unsigned char*>(d1), static_cast<const unsigned char*>(s1), n1);
  DCNN_LAUNCH_CHECK();
}

// fp32 -> [hi | lo | hi] (pattern 0) or [hi | hi | lo] (pattern 1) bf16 rows, 4 channels a thread
__global__ void split3_kernel(const float* __restrict__ in, bf16* __restrict__ out, long rows, int C, int pattern) {
  const int c4n = C / 4;
  const long n = rows * c4n;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const long r = i / c4n;
    const int c = (int)(i - r * c4n) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(in + r * C + c);
    bf16x4 hi, lo;
    for (int k = 0; k < 4; ++k) {
      hi[k] = (bf16)v[k];
      lo[k] = (bf16)(v[k] - (float)hi[k]);
    }
    bf16* o = out + r * 3 * C + c;
    *reinterpret_cast<bf16x4*>(o) = hi;
    *reinterpret_cast<bf16x4*>(o + C) = pattern ? hi : lo;
    *reinterpret_cast<bf16x4*>(o + 2 * C) = pattern ? lo : hi;
  }
}

void split3_bf16(const float* in, bf16* out, long rows, int C, int pattern, hipStream_t s) {
  if (rows <= 0) return;
  if (C % 4 || reinterpret_cast<uintptr_t>(in) % 16 || reinterpret_cast<uintptr_t>(out) % 8)
    throw std::runtime_error("split3_bf16: C % 4 == 0 and aligned buffers only");
  hipLaunchKernelGGL(split3_kernel, dim3(grid_for(rows * (C / 4), 256)), dim3(256), 0, s, in, out, rows, C, pattern);
  DCNN_LAUNCH_CHECK();
}

void grad_pack_bf16(const float* g, bf16* out, long n, float scale, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(grad_pack_kernel, dim3(stream_grid(n)), dim3(256), 0, s, g, out, n, scale);
  DCNN_LAUNCH_CHECK();
}

void grad_sum_chunks_bf16(const bf16* src, int w, long ld, long n, bf16* dst, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(grad_sum_chunks_kernel, dim3(stream_grid(n)), dim3(256), 0, s, src, w, ld, n, dst);
  DCNN_LAUNCH_CHECK();
}

void grad_unpack_bf16(const bf16* in, float* g, long n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(grad_unpack_kernel, dim3(stream_grid(n)), dim3(256), 0, s, in, g, n);
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
