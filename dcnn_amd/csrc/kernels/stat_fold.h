// In-kernel BatchNorm statistics fold: the producing kernel (a conv whose epilogue writes the
// statistics rows of its output / of the fused BatchNorm backward) reduces its own rows, so no
// bn_stat_reduce launch sits between the producer and the BatchNorm that consumes the statistics.
//
// The rows are cut into groups of kStatGroupRows (= the rows bn_stat_reduce merges per level-1
// block). Every row is written with agent-coherent (sc1) stores; when a workgroup has written all
// its rows it waits for them to complete (s_waitcnt vmcnt(0)), and one lane adds one arrival per
// row written to that row's group ticket (agent scope).
// The workgroup whose add completes a group (`arrivals` per row: the column tiles that each write a
// slice of the row) acquires (L2 invalidate), reads the group back with sc1 loads and merges it with bn_stat_reduce's exact
// tree (16-row pairwise trees for 8 virtual waves, then the fixed LDS tree), writing the group's
// level-1 partial (several groups: [parts][3][C], merged by the consumer's read_stats in part
// order) or the finished [2][C] statistics (one group) — bit for bit what the launch produced.
// Tickets are left zeroed for the next launch. No work waits on another workgroup: the last
// arriver simply does more.
//
// Reference parity: the reference reduces BatchNorm statistics in a separate pass
// (src/nn/layers_impl/cuda/batchnorm_ops.cu:297-324).
#pragma once
#include "api.h"
#include "common.h"

namespace dcnn {

constexpr int kStatSC1 = 16;  // cache policy bit: sc1 (agent-coherent)
// (StatFold, kStatGroupRows, stat_fold_groups: api.h)

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stat_rsrc(const float* slab) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(slab), (short)0, 0x7fffffff, 0x00020000);
}
// agent-coherent store of slab element `idx` (the rows another workgroup reads back)
// (the b32 buffer builtins move raw 32-bit words: bit casts, never value conversions)
__device__ __forceinline__ void stat_store_sc1(__amdgpu_buffer_rsrc_t rs, long idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, (unsigned)(idx * 4), 0, kStatSC1);
}
__device__ __forceinline__ float stat_load_sc1(__amdgpu_buffer_rsrc_t rs, unsigned voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, kStatSC1));
}

template <int MODE>
struct FoldAcc {
  float a, b, c;  // MODE 0: (n, mean, M2); MODE 1: (sum a, sum b, -)
  __device__ __forceinline__ FoldAcc merge(const FoldAcc& o) const {
    if constexpr (MODE == 0) {
      const Welford w = welford_merge(Welford{a, b, c}, Welford{o.a, o.b, o.c});
      return FoldAcc{w.n, w.mean, w.m2};
    } else {
      return FoldAcc{a + o.a, b + o.b, 0.f};
    }
  }
};

// LDS bytes the group reduce needs (8 virtual waves x 64 channels)
constexpr int kStatFoldLds = 8 * 64 * 12;

// Reduce group g of a [rows][NV][C] slab (MODE 0: NV = 3 Welford rows; MODE 1: NV = 2 sums) by the
// whole workgroup (4 waves). `lds`: kStatFoldLds bytes, free across this call.
template <int MODE>
__device__ void stat_fold_group(const float* slab, int rows, int C, int g, const StatFold& f, char* lds) {
  constexpr int NV = MODE == 0 ? 3 : 2;
  FoldAcc<MODE>(*red)[64] = reinterpret_cast<FoldAcc<MODE>(*)[64]>(lds);
  // (uniform row conditions only: no per-lane masks held in SGPRs next to a big kernel's state)
  const __amdgpu_buffer_rsrc_t rs = stat_rsrc(slab);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform)
  const int groups = stat_fold_groups(rows);
#pragma unroll 1
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + lane;
    const bool cok = c < C;  // (lanes past C read another row's values and are never written)
    // the channel block's offset rides in the (uniform) soffset, so the row offsets are not loop
    // invariants the compiler would hoist and keep in SGPRs across the channel loop
    const unsigned vo = (unsigned)(lane * 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int vw = w + 4 * h;  // virtual wave: rows [16 vw, 16 vw + 16) of the group
      const int r0 = g * kStatGroupRows + vw * 16;
      // bn_stat_reduce's 16-row pairwise tree as two 8-row trees merged last (the same order)
      FoldAcc<MODE> half[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        FoldAcc<MODE> v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // uniform row offset in soffset; rows past the end (the last group) are zero triples
          const int r = r0 + 8 * q + j;
          const int so = (r * NV * C + c0) * 4;
          if (r < rows) {
            v[j].a = stat_load_sc1(rs, vo, so);
            v[j].b = stat_load_sc1(rs, vo, so + C * 4);
            v[j].c = NV == 3 ? stat_load_sc1(rs, vo, so + 2 * C * 4) : 0.f;
          } else {
            v[j] = FoldAcc<MODE>{0.f, 0.f, 0.f};
          }
        }
#pragma unroll
        for (int s = 1; s < 8; s *= 2)
#pragma unroll
          for (int j = 0; j + s < 8; j += 2 * s) v[j] = v[j].merge(v[j + s]);
        half[q] = v[0];
      }
      red[vw][lane] = half[0].merge(half[1]);
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      __syncthreads();
      if (w < o) red[w][lane] = red[w][lane].merge(red[w + o][lane]);
    }
    __syncthreads();
    if (w == 0 && cok) {
      const FoldAcc<MODE> t = red[0][lane];
      if (groups == 1) {
        if constexpr (MODE == 0) {
          f.out[c] = t.b;
          f.out[C + c] = t.a > 0.f ? t.c / t.a : 0.f;
        } else {
          f.out[c] = t.a;
          f.out[C + c] = t.b;
        }
      } else {
        f.part[((long)g * 3 + 0) * C + c] = t.a;
        f.part[((long)g * 3 + 1) * C + c] = t.b;
        f.part[((long)g * 3 + 2) * C + c] = t.c;
      }
    }
    __syncthreads();
  }
}

// The workgroup has written rows rows_of(0 .. n - 1) (sc1) of a [rows][NV][C] slab: count the
// arrivals and reduce every group this workgroup completed. Every thread of the workgroup calls
// it (it holds barriers); `flags`: n ints of LDS, `lds`: kStatFoldLds bytes.
template <int MODE, class RowOf>
__device__ void stat_fold_arrive(const float* slab, int rows, int C, int n, RowOf rows_of, const StatFold& f,
                                 int* flags, char* lds) {
  // the rows are agent-coherent (sc1) stores — in the memory model, relaxed agent-scope atomic
  // stores — so completing them (s_waitcnt vmcnt(0)) before the arrival orders them; no L2
  // write-back (an agent-scope release fence, buffer_wbl2, per workgroup made gemm_g2 3x slower)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < n; ++k) {
      const int g = rows_of(k) / kStatGroupRows;
      const int rg = min(kStatGroupRows, rows - g * kStatGroupRows);
      const unsigned expect = (unsigned)(rg * f.arrivals);
      const unsigned old = __hip_atomic_fetch_add(f.tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == expect - 1;
      if (last) __hip_atomic_store(f.tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flags[k] = last ? g : -1;
    }
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    const int g = __builtin_amdgcn_readfirstlane(flags[k]);
    if (g >= 0) {
      // acquire: no stale line of the group's rows in this XCD's L2 (buffer_inv sc1)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      stat_fold_group<MODE>(slab, rows, C, g, f, lds);
    }
  }
}
#endif

}  // namespace dcnn
