// In-launch fold of BatchNorm statistics rows (api.h StatFold), shared by the conv epilogues.
//
// A producer writes one statistics row per output tile: forward Welford triples
// [rows][3][N] (count, mean, M2 about the tile's own pivot), backward sums [rows][2][N]
// (sum dy', sum dy' * xhat). Instead of a separate reduce launch (bn_stat_reduce) the tiles of
// a row group count in on a ticket word per (group, 64-column block); the workgroup whose add
// returns the group's last count merges the group's rows for its columns in row order and
// writes the group's partial part[g][3][N] — the [parts][3][N] format the consuming BatchNorm
// kernels merge in their prologue (norm.hip read_stats), or, with a single group, the finished
// [2][N] (mean, biased variance) / (sum a, sum b).
//
// Hand-off without fences (MI355X_MICROARCH.md "Valid forms", row 1): every statistics value is
// stored with an agent-scope (sc1) store, each storing wave drains its stores, one lane adds to
// the ticket after a workgroup barrier, and the merging workgroup reads the rows back with sc1
// loads. Every merge order is fixed (row order within a thread, thread order across), so the
// result does not depend on which workgroup finishes last.
#pragma once
#include "common.h"
#include "api.h"

namespace dcnn {

__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __uint_as_float(
      __hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// stats row store: sc1 when the launch folds (the merging workgroup reads it back), else plain
__device__ __forceinline__ void stat_store(float* p, float v, bool fold) {
  if (fold)
    st_agent(p, v);
  else
    *p = v;
}

// Call after this workgroup stored its statistics row `tm` for columns [n0, n0 + BN) (all 256
// threads, uniform control flow). MODE 0: Welford triples, 1: sums. `scratch`: >= 256 * 3
// floats of LDS that nothing else uses during the call.
template <int MODE, int BN>
__device__ void stat_fold(const float* stats, int N, int tm, int n0, const StatFold& f, float* scratch) {
  static_assert(256 % BN == 0, "column tile must divide the workgroup");
  constexpr int NV = MODE == 0 ? 3 : 2, Q = 256 / BN;
  const int tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row stores have drained
  __syncthreads();
  const int g = tm / f.group;
  const int r0 = g * f.group, r1 = min(f.rows, r0 + f.group);
  volatile int* flag = reinterpret_cast<volatile int*>(scratch);
  if (tid == 0) {
    unsigned* tk = f.tickets + (long)g * (N / 64) + n0 / 64;
    const unsigned old = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(r1 - r0 - 1);
    if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const int last = *flag;
  __syncthreads();
  if (!last) return;
  const int c = tid % BN, q = tid / BN;
  float a = 0.f, b = 0.f, m = 0.f;  // MODE 0: (n, mean, M2); 1: (sum a, sum b)
  // batches of FB rows per thread with every load issued before the first merge (a dependent
  // load-merge chain costs one memory latency per row)
  constexpr int FB = 8;
  for (int rb = r0 + q; rb < r1; rb += FB * Q) {
    float v0[FB], v1[FB], v2[FB];
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int r = rb + j * Q;
      const float* row = stats + (long)(r < r1 ? r : r0) * NV * N + n0 + c;
      v0[j] = ld_agent(row);
      v1[j] = ld_agent(row + N);
      v2[j] = MODE == 0 ? ld_agent(row + 2 * N) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      if (rb + j * Q >= r1) break;
      if (MODE == 0) {
        const Welford w = welford_merge(Welford{a, b, m}, Welford{v0[j], v1[j], v2[j]});
        a = w.n; b = w.mean; m = w.m2;
      } else {
        a += v0[j]; b += v1[j];
      }
    }
  }
  scratch[tid] = a;
  scratch[256 + tid] = b;
  scratch[512 + tid] = m;
  __syncthreads();
  if (q == 0) {
    for (int k = 1; k < Q; ++k) {
      const int o = k * BN + c;
      if (MODE == 0) {
        const Welford w = welford_merge(Welford{a, b, m}, Welford{scratch[o], scratch[256 + o], scratch[512 + o]});
        a = w.n; b = w.mean; m = w.m2;
      } else {
        a += scratch[o]; b += scratch[256 + o];
      }
    }
    if (f.ngroups == 1) {  // finished statistics
      f.part[n0 + c] = MODE == 0 ? b : a;
      f.part[N + n0 + c] = MODE == 0 ? (a > 0.f ? m / a : 0.f) : b;
    } else {
      float* o = f.part + (long)g * 3 * N + n0 + c;
      o[0] = a; o[N] = b; o[2 * N] = m;
    }
  }
}

}  // namespace dcnn
