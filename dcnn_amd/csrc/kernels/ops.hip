// Generic tensor ops of the device-agnostic ops layer (reference include/ops/ops.hpp:17-944,
// CUDA src/ops/cuda/kernels.cu and src/tensor/cuda/tensor_kernels.cu), fp32:
//
// * one vectorised elementwise kernel family (binary / scalar / unary / ternary / axpy) with an
//   op code, 16-byte accesses + scalar tail, grid-stride;
// * deterministic two-pass wave64 reductions (sum, dot, sum of squares, sum of squared
//   differences) into a device scalar — no per-call malloc, no host round trip;
// * Philox-4x32-10 uniform / normal fills (4 values per counter);
// * 64x64 LDS-tiled 2-D transpose and NCHW <-> CNHW permutes;
// * pad / unpad / crop of NCHW tensors.
#include "common.h"
#include "api.h"

namespace dcnn {

enum : int {
  EW_ADD = 0, EW_SUB, EW_MUL, EW_DIV, EW_MIN, EW_MAX, EW_EQ, EW_GT,           // binary / scalar
  EW_SQRT = 16, EW_RSQRT, EW_RCP, EW_ABS, EW_NEG, EW_EXP, EW_LOG, EW_COPY,   // unary
  EW_FMADD = 32, EW_FMSUB, EW_FNMADD,                                        // ternary c = op(a, b, c)
  EW_CLAMP = 48, EW_SUB_MUL, EW_MUL_ADD                                      // (a, s0, s1)
};

__device__ __forceinline__ float ew2(int op, float a, float b) {
  switch (op) {
    case EW_ADD: return a + b;
    case EW_SUB: return a - b;
    case EW_MUL: return a * b;
    case EW_DIV: return a / b;
    case EW_MIN: return fminf(a, b);
    case EW_MAX: return fmaxf(a, b);
    case EW_EQ: return a == b ? 1.f : 0.f;
    default: return a > b ? 1.f : 0.f;
  }
}

__device__ __forceinline__ float ew1(int op, float a, float s0, float s1) {
  switch (op) {
    case EW_SQRT: return sqrtf(a);
    case EW_RSQRT: return rsqrtf(a);
    case EW_RCP: return 1.f / a;
    case EW_ABS: return fabsf(a);
    case EW_NEG: return -a;
    case EW_EXP: return __expf(a);
    case EW_LOG: return __logf(a);
    case EW_COPY: return a;
    case EW_CLAMP: return fminf(fmaxf(a, s0), s1);
    case EW_SUB_MUL: return (a - s0) * s1;
    case EW_MUL_ADD: return a * s0 + s1;
    default: return a;
  }
}

// mode 0: c = op(a, b)   mode 1: c = op(a, s0)   mode 2: c = unary(a)   mode 3: c = ternary(a, b, c)
// mode 4: c += s0 * a (axpy)
__global__ void ew_kernel(int mode, int op, const float* __restrict__ a, const float* __restrict__ b, float* c, long n,
                          float s0, float s1) {
  const long n4 = n >> 2;
  const long stride = (long)gridDim.x * blockDim.x;
  const bool al = ((((uintptr_t)a) | ((uintptr_t)c) | (b ? (uintptr_t)b : 0)) & 15) == 0;
  auto one = [&](float x, float y, float z) -> float {
    switch (mode) {
      case 0: return ew2(op, x, y);
      case 1: return ew2(op, x, s0);
      case 2: return ew1(op, x, s0, s1);
      case 3: return op == EW_FMADD ? x * y + z : (op == EW_FMSUB ? x * y - z : -(x * y) + z);
      default: return z + s0 * x;
    }
  };
  long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (al) {
    for (long i = i0; i < n4; i += stride) {
      const float4 x = reinterpret_cast<const float4*>(a)[i];
      const float4 y = b ? reinterpret_cast<const float4*>(b)[i] : make_float4(0, 0, 0, 0);
      const float4 z = (mode >= 3) ? reinterpret_cast<const float4*>(c)[i] : make_float4(0, 0, 0, 0);
      reinterpret_cast<float4*>(c)[i] = make_float4(one(x.x, y.x, z.x), one(x.y, y.y, z.y), one(x.z, y.z, z.z),
                                                    one(x.w, y.w, z.w));
    }
    for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
      c[i] = one(a[i], b ? b[i] : 0.f, mode >= 3 ? c[i] : 0.f);
  } else {
    for (long i = i0; i < n; i += stride) c[i] = one(a[i], b ? b[i] : 0.f, mode >= 3 ? c[i] : 0.f);
  }
}

void elementwise(int mode, int op, const float* a, const float* b, float* c, long n, float s0, float s1, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ew_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, s, mode, op, a, b, c, n, s0, s1);
}

// ---- reductions: partial per block, then one block finishes (deterministic)
__global__ void reduce_partial_kernel(int op, const float* __restrict__ a, const float* __restrict__ b, long n,
                                      float* part) {
  __shared__ float sh[32];
  float acc = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = a[i];
    switch (op) {
      case 0: acc += x; break;                                  // sum
      case 1: acc += x * b[i]; break;                           // dot
      case 2: acc += x * x; break;                              // norm squared
      default: { const float d = x - b[i]; acc += d * d; }      // sum of squared differences
    }
  }
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void reduce_final_kernel(const float* part, int nb, float* out) {
  __shared__ float sh[32];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) out[0] = acc;
}

void reduce(int op, const float* a, const float* b, long n, float* workspace, float* out, hipStream_t s) {
  const int nb = grid_for(n, 256, 1024);
  hipLaunchKernelGGL(reduce_partial_kernel, dim3(nb), dim3(256), 0, s, op, a, b, n, workspace);
  hipLaunchKernelGGL(reduce_final_kernel, dim3(1), dim3(256), 0, s, workspace, nb, out);
}

// ---- Philox fills
__global__ void fill_random_kernel(float* out, long n, uint64_t seed, float a, float b, int normal) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q * 4 < n; q += (long)gridDim.x * blockDim.x) {
    const uint4 r = Philox::gen(seed, (uint64_t)q);
    float v[4];
    if (normal) {  // Box-Muller on two pairs: mean a, std b
      const float u1 = fmaxf(Philox::u01(r.x), 1e-12f), u2 = Philox::u01(r.y);
      const float u3 = fmaxf(Philox::u01(r.z), 1e-12f), u4 = Philox::u01(r.w);
      const float r1 = sqrtf(-2.f * __logf(u1)), r2 = sqrtf(-2.f * __logf(u3));
      v[0] = r1 * __cosf(6.28318530718f * u2);
      v[1] = r1 * __sinf(6.28318530718f * u2);
      v[2] = r2 * __cosf(6.28318530718f * u4);
      v[3] = r2 * __sinf(6.28318530718f * u4);
      for (int k = 0; k < 4; ++k) v[k] = a + b * v[k];
    } else {  // uniform [a, b)
      v[0] = a + (b - a) * Philox::u01(r.x);
      v[1] = a + (b - a) * Philox::u01(r.y);
      v[2] = a + (b - a) * Philox::u01(r.z);
      v[3] = a + (b - a) * Philox::u01(r.w);
    }
    for (int k = 0; k < 4; ++k)
      if (q * 4 + k < n) out[q * 4 + k] = v[k];
  }
}

void fill_random(float* out, long n, uint64_t seed, float a, float b, int normal, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_random_kernel, dim3(grid_for((n + 3) / 4, 256)), dim3(256), 0, s, out, n, seed, a, b, normal);
}

// ---- transposes
// out[c][r] = in[r][c] for a batch of B matrices (rows x cols), 64x64 LDS tiles (+1 pad)
__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, int rows, int cols) {
  __shared__ float tile[64][65];
  const long boff = (long)blockIdx.z * rows * cols;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 64 x 4
  for (int j = ty; j < 64; j += 4) {
    const int r = r0 + j, c = c0 + tx;
    tile[j][tx] = (r < rows && c < cols) ? in[boff + (long)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 64; j += 4) {
    const int c = c0 + j, r = r0 + tx;
    if (c < cols && r < rows) out[boff + (long)c * rows + r] = tile[tx][j];
  }
}

void transpose_batched(const float* in, float* out, int batch, int rows, int cols, hipStream_t s) {
  dim3 g((cols + 63) / 64, (rows + 63) / 64, batch);
  hipLaunchKernelGGL(transpose_kernel, g, dim3(256), 0, s, in, out, rows, cols);
}

// the same for 16-bit elements (bf16 activations): NCHW <-> NHWC around the NCHW-order Flatten of
// a spatial map (per image [C][HW] <-> [HW][C])
__global__ void transpose16_kernel(const unsigned short* __restrict__ in, unsigned short* __restrict__ out, int rows,
                                   int cols) {
  __shared__ unsigned short tile[64][66];
  const long boff = (long)blockIdx.z * rows * cols;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int j = ty; j < 64; j += 4) {
    const int r = r0 + j, c = c0 + tx;
    tile[j][tx] = (r < rows && c < cols) ? in[boff + (long)r * cols + c] : (unsigned short)0;
  }
  __syncthreads();
  for (int j = ty; j < 64; j += 4) {
    const int c = c0 + j, r = r0 + tx;
    if (c < cols && r < rows) out[boff + (long)c * rows + r] = tile[tx][j];
  }
}

void transpose_batched16(const void* in, void* out, int batch, int rows, int cols, hipStream_t s) {
  dim3 g((cols + 63) / 64, (rows + 63) / 64, batch);
  hipLaunchKernelGGL(transpose16_kernel, g, dim3(256), 0, s, (const unsigned short*)in, (unsigned short*)out, rows,
                     cols);
  DCNN_LAUNCH_CHECK();
}

// ---- strided row copy / accumulate: dst[r][c] (+)= src[r][c], c < cols, row pitches lds / ldd
// (channel-padded conv operands: the RGB-like conv's bf16 weight rows into an 8-channel padded
// operand, and its padded weight gradient back into the real channels). kind: 0 bf16 -> bf16
// copy, 1 fp32 -> fp32 accumulate.
template <class TI, class TO, bool ACC>
__global__ void rows_copy_kernel(const TI* __restrict__ src, int lds, TO* __restrict__ dst, int ldd, long rows,
                                 int cols) {
  const long total = rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols;
    const int c = (int)(i - r * cols);
    const float v = to_f(src[r * lds + c]);
    TO* d = dst + r * ldd + c;
    *d = from_f<TO>(ACC ? to_f(*d) + v : v);
  }
}

void rows_copy(int kind, const void* src, int lds, void* dst, int ldd, long rows, int cols, hipStream_t s) {
  const int g = grid_for(rows * cols, 256);
  if (kind == 0)
    hipLaunchKernelGGL((rows_copy_kernel<bf16, bf16, false>), dim3(g), dim3(256), 0, s, (const bf16*)src, lds,
                       (bf16*)dst, ldd, rows, cols);
  else if (kind == 1)
    hipLaunchKernelGGL((rows_copy_kernel<float, float, true>), dim3(g), dim3(256), 0, s, (const float*)src, lds,
                       (float*)dst, ldd, rows, cols);
  else
    throw std::runtime_error("rows_copy: bad kind");
  DCNN_LAUNCH_CHECK();
}

// NCHW [N][C][HW] <-> CNHW [C][N][HW]: a permutation of HW-contiguous rows
__global__ void nchw_cnhw_kernel(const float* __restrict__ in, float* __restrict__ out, int N, int C, int HW,
                                 int to_cnhw) {
  const long total = (long)N * C * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int p = (int)(i % HW);
    const long r = i / HW;
    // i indexes the *output*
    if (to_cnhw) {
      const int n = (int)(r % N), c = (int)(r / N);
      out[i] = in[((long)n * C + c) * HW + p];
    } else {
      const int c = (int)(r % C), n = (int)(r / C);
      out[i] = in[((long)c * N + n) * HW + p];
    }
  }
}

void nchw_cnhw(const float* in, float* out, int N, int C, int HW, int to_cnhw, hipStream_t s) {
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(nchw_cnhw_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, in, out, N, C, HW, to_cnhw);
}

// ---- pad / unpad (crop) of NCHW: out[n][c][y][x] = in[n][c][y - top][x - left] (0 outside)
__global__ void pad_crop_kernel(const float* __restrict__ in, float* __restrict__ out, int NC, int H, int W, int OH,
                                int OW, int top, int left, float value) {
  const long total = (long)NC * OH * OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % OW);
    const long r = i / OW;
    const int y = (int)(r % OH);
    const long nc = r / OH;
    const int sy = y - top, sx = x - left;
    out[i] = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? in[(nc * H + sy) * W + sx] : value;
  }
}

void pad_crop(const float* in, float* out, int NC, int H, int W, int OH, int OW, int top, int left, float value,
              hipStream_t s) {
  const long total = (long)NC * OH * OW;
  hipLaunchKernelGGL(pad_crop_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, in, out, NC, H, W, OH, OW, top,
                     left, value);
}

}  // namespace dcnn
