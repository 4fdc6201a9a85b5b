// Shared CDNA4 (gfx950) device helpers for the dcnn_amd kernel library.
// Wave64 everywhere: reductions use 64-lane shuffles (reference defect G16 hard-coded 32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>
#include <type_traits>

#ifndef DCNN_BF16_DEFINED
#define DCNN_BF16_DEFINED
#endif
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DCNN_HIP_CHECK(expr)                                                                   \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +   \
                               __FILE__ + ":" + std::to_string(__LINE__));                     \
  } while (0)

#define DCNN_LAUNCH_CHECK() DCNN_HIP_CHECK(hipGetLastError())

namespace dcnn {

constexpr int kWave = 64;

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- kernel-argument prefetch ---------------------------------------------------------------
// Kernels with more arguments than their SGPR budget holds get their argument loads sunk to the
// first uses, one scalar-load round trip to memory per group (hconv3: five serialised groups in
// the prologue). One batch of loads touching every 64-byte line of the argument segment, issued
// first and waited for once, turns those later loads into scalar-cache hits.
template <int BYTES>
__device__ __forceinline__ void prefetch_kernargs() {
  typedef const __attribute__((address_space(4))) unsigned karg_u32;
  karg_u32* k = (karg_u32*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned d = 0;
#pragma unroll
  for (int o = 0; o < BYTES; o += 64) d ^= __builtin_nontemporal_load(k + o / 4);
  asm volatile("" ::"s"(d));
}

// ---- opaque 16-byte direct-to-LDS loads ------------------------------------------------------
// The compiler's wait-count pass cannot tell which LDS bytes a builtin LDS-DMA load writes, so it
// puts `s_waitcnt vmcnt(0)` in front of every later ds_read_b64_tr_b16 — which serialises a
// double-buffered loop (the prefetch of tile k+1 must land before tile k is read). Issued from
// inline asm the DMA is invisible to that pass; the kernels order it themselves with an explicit
// `s_waitcnt vmcnt(0)` + barrier before the buffer is read.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 raw_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = (int)(uint32_t)a;
  r[1] = (int)((a >> 32) & 0xffff);  // stride 0
  r[2] = (int)bytes;                 // num_records: offsets >= bytes read zeros
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void glds16_opaque(i32x4 rsrc, const char* lds, unsigned voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

// Block-wide sum for blockDim.x <= 1024 (wave64). `sh` needs >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}

// ---- BatchNorm statistics partials (deterministic, cancellation-free) ----------------------
// Every producer of forward BatchNorm statistics writes, per tile and channel, the triple
// (count, mean, M2 = sum (x - mean)^2) into a slab [tiles][3][C]. Within a tile the sums are
// taken about a pivot (a value of the tile itself), so E[x^2] - mean^2 cancellation never
// happens; tiles are combined with Chan's pairwise update in a fixed order (bn_stat_reduce).
struct Welford {
  float n, mean, m2;
};
__device__ __forceinline__ Welford welford_merge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (b.n <= 0.f) return a;
  if (a.n <= 0.f) return b;
  const float d = b.mean - a.mean, f = b.n / n;
  return Welford{n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}
// tile triple from pivot-shifted sums: s1 = sum (x - p), s2 = sum (x - p)^2 over n values
__device__ __forceinline__ Welford welford_from_shifted(float n, float p, float s1, float s2) {
  if (n <= 0.f) return Welford{0.f, 0.f, 0.f};
  const float d = s1 / n;
  return Welford{n, p + d, fmaxf(s2 - s1 * d, 0.f)};
}
__device__ __forceinline__ void store_welford(float* slab, long tile, int C, int c, Welford w) {
  slab[(tile * 3 + 0) * C + c] = w.n;
  slab[(tile * 3 + 1) * C + c] = w.mean;
  slab[(tile * 3 + 2) * C + c] = w.m2;
}

// 8 x bf16 <-> 8 x f32 through one 16-byte access.
struct alignas(16) Pack8 {
  uint4 u;
};
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const bf16* b = reinterpret_cast<const bf16*>(&u);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 u;
  bf16* b = reinterpret_cast<bf16*>(&u);
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (bf16)f[i];
  return u;
}

// Philox-4x32-10 counter RNG (stateless: dropout masks are regenerated in backward).
struct Philox {
  __device__ __forceinline__ static uint4 gen(uint64_t seed, uint64_t ctr) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0x6a09e667u, c3 = 0xbb67ae85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      uint64_t p0 = (uint64_t)0xD2511F53u * c0;
      uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
      uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
      uint32_t n1 = (uint32_t)p1;
      uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
      uint32_t n3 = (uint32_t)p0;
      c0 = n0;
      c1 = n1;
      c2 = n2;
      c3 = n3;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
  __device__ __forceinline__ static float u01(uint32_t x) {
    return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f);
  }
};

// Division by a run-time invariant divisor d >= 1 (Granlund-Montgomery): q = (umulhi(n, mul) + n)
// >> shr, exact for n < 2^31. The launcher builds it once; in the kernel it is a multiply-high, an
// add and a shift (scalar or vector) instead of the ~40-instruction reciprocal sequence of a
// plain run-time division.
struct FastDiv {
  unsigned mul, shr, d;
};
inline FastDiv make_fastdiv(unsigned d) {
  unsigned l = 0;
  while ((1ull << l) < d) ++l;
  const unsigned long long m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{(unsigned)m, l, d};
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shr; }

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
inline int grid_for(long n, int block, int cap = 2048 * 4) {
  long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dcnn
