// Implicit-GEMM convolution v2 for CDNA4 (gfx950): direct-to-LDS gather + MFMA 16x16x32 bf16.
//
// One generic "gathered NT GEMM" covers conv forward, conv dgrad (phase-decomposed for strided
// convs so no MFMA work is spent on structurally-zero taps) and dense layers:
//
//   C[m][n] = sum_{t < ntaps, c < Cs} Src[img(m), gy(m)*SY + dy[t], gx(m)*SX + dx[t], c] * B[n][tapB[t] + c]
//
// * Src is an NHWC bf16 tensor; every 16-byte chunk of a tile row is fetched with
//   `buffer_load_dwordx4 ... lds` straight into LDS (no VGPR staging, no ds_write). Padding /
//   out-of-image taps are handled by the buffer descriptor's range check: an invalid chunk gets an
//   out-of-range offset and the hardware writes zeros.
// * Per GEMM row the validity of every tap is precomputed once into a 64-bit mask, so the K loop
//   costs ~3 VALU per 16-byte chunk (mask test, select, add).
// * LDS tiles are XOR-swizzled through the *source* address (glds writes lane-linear), read with
//   conflict-free ds_read_b128; 2-stage pipeline: tile k+1 in flight while tile k is multiplied.
// * Epilogue: bias added in registers, tile staged through LDS as bf16, then 16-byte coalesced
//   stores with fused residual add, ReLU and per-channel (sum, sum^2) BatchNorm partials; the
//   output row mapping supports the strided scatter of a dgrad phase.
//
// The weight-gradient kernel (tn2) uses the same loader on both operands (pixels = K) and
// ds_read_b64_tr_b16 transposed fragment reads; split-K partials go to an fp32 slab.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "api.h"

namespace dcnn {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int xcd_remap2(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t rsrc, char* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

constexpr unsigned kOOB = 0x80000000u;  // any offset >= num_records reads zeros

// n / d for n < 2^31 with G2Args' multiply-shift reciprocal {mul, shr, d} (common.h FastDiv)
__device__ __forceinline__ unsigned g2_div(int n, const unsigned* f) {
  return fdiv((unsigned)n, FastDiv{f[0], f[1], f[2]});
}

// ---------------------------------------------------------------------------------------------
// gathered NT GEMM
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, bool UNI, int NST>
struct G2 {
  static constexpr int CPR = BK / 8;                 // 16-B chunks per LDS row
  static constexpr int RPI = 64 / CPR;               // rows covered by one wave-instruction (1 KiB)
  static constexpr int RPB = 256 / (BK * 2);         // rows per 256-B bank row
  static constexpr int A_INS = BM / RPI / 4;         // glds instructions per wave for A
  static constexpr int B_INS = BN / RPI / 4;
  static constexpr int TM = BM / 32, TN = BN / 32;   // 16x16 subtiles per wave (2x2 waves)
  static constexpr int STAGE = (BM + BN) * BK * 2;
  static constexpr int EPI_PITCH = BN * 2 + 16;      // bf16 staging row pitch (bytes)
  static constexpr int LDS = (NST * STAGE > BM * EPI_PITCH) ? NST * STAGE : BM * EPI_PITCH;
  static constexpr int INS = A_INS + B_INS;          // glds instructions per wave per stage
  __device__ static __forceinline__ int swz(int row) { return (row / RPB) % CPR; }
  __device__ static __forceinline__ int off(int row, int ch) { return row * (BK * 2) + ((ch ^ swz(row)) << 4); }
};

// ---- epilogue 2 (shared by the GEMM and its split-K epilogue kernel): the bf16 tile staged in
// LDS ([BM][EPI_PITCH]) -> 16-byte rows to global (+residual, ReLU, backward-BN mask) and the
// BatchNorm statistics rows of the stored values. All 256 threads; holds barriers.
template <int BM, int BN, int EPI_PITCH>
__device__ __forceinline__ void g2_epilogue2(const G2Args& p, char* smem, int m0, int n0, int tm, int mcls, int ory,
                                             int orx) {
  const int tid = threadIdx.x;
  // ---- epilogue 2: 16-byte rows -> global (+residual, ReLU, BN partial stats) ----
  constexpr int CG = BN / 8;           // column groups of 8
  constexpr int RSTEP = 256 / CG;      // rows handled concurrently
  const int cg = tid % CG, r0 = tid / CG;
  const int ncol = n0 + cg * 8;
  const bool col_ok = ncol < p.N;      // N % 8 == 0 for this kernel
  float s[8], q[8], mu[8], is[8], pv[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) s[v] = q[v] = mu[v] = is[v] = pv[v] = 0.f;
  const bool bnb = p.bnb.x != nullptr;  // backward-BN fusion (api.h BnbArgs)
  if (bnb && col_ok) {
#pragma unroll
    for (int v = 0; v < 8; ++v) { mu[v] = p.bnb.mean[ncol + v]; is[v] = p.bnb.istd[ncol + v]; }
  }
  // forward statistics about a pivot (tile row 0, always a valid row): (count, mean, M2) triples
  float piv_col = 0.f;
  if (p.stats && !bnb) {
    unpack8(*reinterpret_cast<const uint4*>(smem + cg * 16), pv);
    if (tid < BN) piv_col = (float)*reinterpret_cast<const bf16*>(smem + tid * 2);
  }
  const int ghw = p.GH * p.GW;
  auto orow_of = [&](int row) {
    const int ml = m0 + row - mcls;
    const int img = (int)g2_div(ml, p.fd_ghw), rem = ml - img * ghw;
    const int gy = (int)g2_div(rem, p.fd_gw), gx = rem - gy * p.GW;
    return ((long)img * p.OH + gy * p.OSY + ory) * p.OW + gx * p.OSX + orx;
  };
  // every row's operands are loaded before the first store: a load's wait also waits for every
  // older store, and one latency per tile instead of one per row matters at 2 waves per SIMD
  const bool has_res = p.residual != nullptr, has_y = bnb && p.bnb.y != nullptr, has_x = bnb && p.stats;
  constexpr int NR = BM / RSTEP;       // rows per thread
  uint4 c_res[NR], c_y[NR], c_x[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    c_res[i] = c_y[i] = c_x[i] = uint4{0u, 0u, 0u, 0u};
    const int row = r0 + i * RSTEP;
    if (m0 + row >= p.M || !col_ok) continue;
    const long o = orow_of(row) * p.ldc + ncol;
    if (has_res) c_res[i] = *reinterpret_cast<const uint4*>(p.residual + o);
    if (has_y) c_y[i] = *reinterpret_cast<const uint4*>(p.bnb.y + o);
    if (has_x) c_x[i] = *reinterpret_cast<const uint4*>(p.bnb.x + o);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int row = r0 + i * RSTEP;
    const int m = m0 + row;
    if (m < p.M && col_ok) {
      const long orow = orow_of(row);
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(smem + row * EPI_PITCH + cg * 16), f);
      if (has_res) {
        float rr[8];
        unpack8(c_res[i], rr);
#pragma unroll
        for (int v = 0; v < 8; ++v) f[v] += rr[v];
      }
      if (p.relu) {
#pragma unroll
        for (int v = 0; v < 8; ++v) f[v] = fmaxf(f[v], 0.f);
      }
      if (has_y) {
        float yo[8];
        unpack8(c_y[i], yo);
#pragma unroll
        for (int v = 0; v < 8; ++v) f[v] = yo[v] > 0.f ? f[v] : 0.f;
      }
      const uint4 o = pack8(f);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p.C) + orow * p.ldc + ncol) = o;
      if (p.stats) {
        float g[8];
        unpack8(o, g);
        if (bnb) {
          float xv[8];
          unpack8(c_x[i], xv);
#pragma unroll
          for (int v = 0; v < 8; ++v) { s[v] += g[v]; q[v] += g[v] * (xv[v] - mu[v]) * is[v]; }
        } else {
#pragma unroll
          for (int v = 0; v < 8; ++v) { const float d = g[v] - pv[v]; s[v] += d; q[v] += d * d; }
        }
      }
    }
  }
  if (p.stats) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [RSTEP][2][BN]
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      red[(r0 * 2 + 0) * BN + cg * 8 + v] = s[v];
      red[(r0 * 2 + 1) * BN + cg * 8 + v] = q[v];
    }
    __syncthreads();
    if (bnb) {  // backward: plain sums [tiles][2][N]
      for (int c = tid; c < 2 * BN; c += 256) {
        const int which = c / BN, cc = c % BN;
        if (n0 + cc < p.N) {
          float a = 0.f;
          for (int k = 0; k < RSTEP; ++k) a += red[(k * 2 + which) * BN + cc];
          p.stats[((long)tm * 2 + which) * p.N + n0 + cc] = a;
        }
      }
    } else if (tid < BN && n0 + tid < p.N) {  // forward: Welford triple [tiles][3][N]
      float a = 0.f, b = 0.f;
      for (int k = 0; k < RSTEP; ++k) { a += red[(k * 2 + 0) * BN + tid]; b += red[(k * 2 + 1) * BN + tid]; }
      const float cnt = (float)min(BM, p.M - m0);
      store_welford(p.stats, tm, p.N, n0 + tid, welford_from_shifted(cnt, piv_col, a, b));
    }
  }
}

// SPLIT: the split-K instance (gemm_g2() on long-K 1x1 GEMMs: workgroup = (tile, K slice), fp32
// partial tiles out, g2_splitk_epi_kernel runs the epilogue). A separate instance: the slice decode
// and the partial store cost the plain instances ~50 VGPRs and an occupancy step.
template <int BM, int BN, int BK, bool UNI, int NST, bool SPLIT = false>
__global__ void __launch_bounds__(256, 2) gemm_g2_kernel(G2Args p) {
  prefetch_kernargs<sizeof(G2Args)>();
  using T = G2<BM, BN, BK, UNI, NST>;
  __shared__ __attribute__((aligned(16))) char smem[T::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int lt_all = xcd_remap2(blockIdx.x, gridDim.x);
  // split-K (plain 1x1 GEMMs with long K on small grids, gemm_g2()): workgroup = (tile, K slice);
  // the slices of a tile are neighbours in the remapped order (one XCD's L2 holds the tile's B)
  const int ks = SPLIT ? p.ksplit : 1;
  const int lt = SPLIT ? lt_all / ks : lt_all, kslice = SPLIT ? lt_all - lt * ks : 0;
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  // row class of this tile (grouped strided-dgrad phases; one class otherwise). The classes are
  // interleaved tile row by tile row: each XCD's contiguous share of the remapped grid holds every
  // phase of the same pixels (the dY rows they share stay in that XCD's L2, and the 4-tap class
  // is not one XCD's tail)
  const int cls = p.ncls > 1 ? tm % p.ncls : 0;
  const int m0 = p.ncls > 1 ? cls * p.cls_rows + (tm / p.ncls) * BM : tm * BM, n0 = tn * BN;
  const int mcls = cls * p.cls_rows;                 // first row of the class
  const int ct0 = p.cls_t0[cls], ntp = p.cls_nt[cls];
  const int ory = p.cls_ory[cls], orx = p.cls_orx[cls];

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);
  if (p.zero_ptr && blockIdx.x == 0) {
    for (int i = tid; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the glds counting below exact
  }

  // ---- per-lane A rows: pixel base offset + tap-validity mask (fixed over the K loop) ----
  const int ch = lane % T::CPR;           // this lane's physical chunk slot within a row
  unsigned a_base[T::A_INS];
  uint64_t a_mask[T::A_INS];
  int a_lch[T::A_INS];                    // logical chunk fetched by this lane (source-side swizzle)
#pragma unroll
  for (int i = 0; i < T::A_INS; ++i) {
    const int row = (wid * T::A_INS + i) * T::RPI + lane / T::CPR;
    a_lch[i] = ch ^ T::swz(row);
    const int m = m0 + row;
    uint64_t mask = 0;
    unsigned base = 0;
    if (m < p.M) {
      const int ml = m - mcls;
      const int img = (int)g2_div(ml, p.fd_ghw), rem = ml - img * p.GH * p.GW;
      const int gy = (int)g2_div(rem, p.fd_gw), gx = rem - gy * p.GW;
      const int y0 = gy * p.SY, x0 = gx * p.SX;
      base = (unsigned)((((long)img * p.H + y0) * p.W + x0) * p.Cs * 2);
      for (int t = 0; t < ntp; ++t) {
        const int sy = y0 + p.tap_dy[ct0 + t], sx = x0 + p.tap_dx[ct0 + t];
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W) mask |= (1ull << t);
      }
    }
    a_base[i] = base;
    a_mask[i] = mask;
  }
  unsigned b_base[T::B_INS];
  bool b_ok[T::B_INS];
  int b_lch[T::B_INS];
#pragma unroll
  for (int i = 0; i < T::B_INS; ++i) {
    const int row = (wid * T::B_INS + i) * T::RPI + lane / T::CPR;
    b_lch[i] = ch ^ T::swz(row);
    const int n = n0 + row;
    b_ok[i] = n < p.N;
    b_base[i] = (unsigned)((long)n * p.ldb * 2);
  }

  // this class's tap table in VGPR lanes (ntaps <= 64 = one wave): lane t holds tap t's source
  // offset and weight column, so a K-step's uniform tap reads its entries with v_readlane — no
  // scalar-memory round trip (and s_waitcnt lgkmcnt(0), which also drains the MFMA operands' LDS
  // reads) per glds instruction in the K loop
  const int tab_src = lane < ntp ? p.tap_srcoff[ct0 + lane] : 0;
  const int tab_b = lane < ntp ? p.tap_b[ct0 + lane] : 0;
  // UNI: the K-steps are staged in order, BK apart, so the (tap, channel) of the next stage is a
  // uniform counter pair (no per-stage integer division)
  int st_t = 0, st_c = 0;

  auto stage = [&](int buf, int k0) {
    char* As = smem + buf * T::STAGE;
    char* Bs = As + BM * BK * 2;
    if constexpr (UNI) {
      const int t = st_t, c0 = st_c;
      st_c += BK;
      if (st_c >= p.Cs) { st_c -= p.Cs; ++st_t; }
      const bool tok = t < ntp;
      const int tl = tok ? t : 0;
      const int src = __builtin_amdgcn_readlane(tab_src, tl), tb = __builtin_amdgcn_readlane(tab_b, tl);
#pragma unroll
      for (int i = 0; i < T::A_INS; ++i) {
        const int c = c0 + a_lch[i] * 8;
        const bool ok = tok && c < p.Cs && ((a_mask[i] >> tl) & 1ull);
        const unsigned voff = ok ? a_base[i] + (unsigned)(src * 2 + c * 2) : kOOB;
        glds16(rsA, As + (wid * T::A_INS + i) * 1024, voff);
      }
#pragma unroll
      for (int i = 0; i < T::B_INS; ++i) {
        const int c = c0 + b_lch[i] * 8;
        const bool ok = b_ok[i] && tok && c < p.Cs;
        const unsigned voff = ok ? b_base[i] + (unsigned)((tb + c) * 2) : kOOB;
        glds16(rsB, Bs + (wid * T::B_INS + i) * 1024, voff);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < T::A_INS; ++i) {
      const int k = k0 + a_lch[i] * 8;
      const int t = k / p.Cs, c = k - t * p.Cs;
      const bool ok = t < ntp && c < p.Cs && ((a_mask[i] >> t) & 1ull);
      const unsigned voff = ok ? a_base[i] + (unsigned)(p.tap_srcoff[ct0 + t] * 2 + c * 2) : kOOB;
      glds16(rsA, As + (wid * T::A_INS + i) * 1024, voff);
    }
#pragma unroll
    for (int i = 0; i < T::B_INS; ++i) {
      const int k = k0 + b_lch[i] * 8;
      const int t = k / p.Cs, c = k - t * p.Cs;
      const bool ok = b_ok[i] && t < ntp && c < p.Cs;
      const unsigned voff = ok ? b_base[i] + (unsigned)((p.tap_b[ct0 + t] + c) * 2) : kOOB;
      glds16(rsB, Bs + (wid * T::B_INS + i) * 1024, voff);
    }
  };

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int K = ntp * p.Cs;
  const int nk_all = (K + BK - 1) / BK;
  // this workgroup's K-steps [kb, kb + nk) (all of them without split-K)
  const int kb = SPLIT ? (int)((long)nk_all * kslice / ks) : 0;
  const int nk = SPLIT ? (int)((long)nk_all * (kslice + 1) / ks) - kb : nk_all;
  if constexpr (UNI && SPLIT) {  // (the stage counters start at the slice's first K-step)
    const int k0 = kb * BK;
    st_t = k0 / p.Cs;
    st_c = k0 - st_t * p.Cs;
  }
  auto compute = [&](int buf) {
    const char* As = smem + buf * T::STAGE;
    const char* Bs = As + BM * BK * 2;
    // every fragment of the K-step is read up front (one LDS latency per stage, not one per 32-wide
    // slice: the second slice's reads are in flight while the first slice's MFMAs issue)
    constexpr int KK = BK / 32;
    bf16x8 a[KK][T::TM], b[KK][T::TN];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int c = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
        a[kk][i] = *reinterpret_cast<const bf16x8*>(As + T::off(wm * (BM / 2) + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
        b[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + T::off(wn * (BN / 2) + j * 16 + (lane & 15), c));
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  const int kofs = kb * BK;
  if constexpr (NST == 2) {
    stage(0, kofs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage(cur ^ 1, kofs + (kt + 1) * BK);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // 3-buffer ring: tile k+2 is issued while tile k is multiplied, so every load has two
    // MFMA phases to land. Only counted vmcnt waits (the newest stage stays in flight across
    // the barrier) and raw s_barrier, which unlike __syncthreads() does not drain the
    // outstanding LDS-DMA.
    stage(0, kofs);
    if (nk > 1) {
      stage(1, kofs + BK);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::INS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 2 < nk;
      if (more) stage(cur == 0 ? 2 : cur - 1, kofs + (kt + 2) * BK);
      compute(cur);
      if (more) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(T::INS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      cur = cur == 2 ? 0 : cur + 1;
    }
  }

  if constexpr (SPLIT) {
    // fp32 partial tile of this K slice -> kpart[slice][M][N] (the epilogue kernel sums the
    // slices in order and runs the epilogue, g2_splitk_epi_kernel)
    float* out = p.kpart + (long)kslice * p.M * p.N;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j) {
        const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
          if (m < p.M && n < p.N) out[(long)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  // ---- epilogue 1: acc (+bias) -> bf16 LDS tile [BM][BN] ----
#pragma unroll
  for (int j = 0; j < T::TN; ++j) {
    const int col = wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = (p.bias && n0 + col < p.N) ? p.bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        *reinterpret_cast<bf16*>(smem + row * T::EPI_PITCH + col * 2) = (bf16)(acc[i][j][r] + bv);
      }
  }
  __syncthreads();
  g2_epilogue2<BM, BN, T::EPI_PITCH>(p, smem, m0, n0, tm, mcls, ory, orx);
}

constexpr int kG2MaxSplit = 8;  // K slices of the split-K path at most

// split-K epilogue (gemm_g2 with ksplit > 1): output tile (tm, tn) = the fixed-order sum of the
// K slices' fp32 partials (+bias), staged as the bf16 tile epilogue 1 would have staged, then the
// GEMM's own epilogue 2 (residual, ReLU, backward-BN mask, statistics rows) — the same statistics
// row per BM-row tile as the unsplit kernel, so the consumers see the same layout
template <int BM, int BN>
__global__ void __launch_bounds__(256, 2) g2_splitk_epi_kernel(G2Args p) {
  prefetch_kernargs<sizeof(G2Args)>();
  constexpr int EPI_PITCH = BN * 2 + 16;
  constexpr int RSTEP = 256 / (BN / 8);
  constexpr int L1 = BM * EPI_PITCH, L2 = RSTEP * 2 * BN * 4;
  constexpr int LDS = L1 > L2 ? L1 : L2;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int tid = threadIdx.x;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int lt = xcd_remap2(blockIdx.x, gridDim.x);
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  constexpr int C4 = BN / 4, RS = 256 / C4;  // 4 columns per thread, RS rows at a time
  const int c4 = tid % C4, rr = tid / C4;
  const int n = n0 + c4 * 4;
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && n < p.N) {
#pragma unroll
    for (int v = 0; v < 4; ++v) bv[v] = p.bias[n + v];
  }
  const long slice = (long)p.M * p.N;
  const int ks = p.ksplit;  // (<= kG2MaxSplit)
  // every slice's partial of two rows is loaded before the first add (one memory latency per
  // row pair, not one per slice), then summed in slice order (deterministic)
  static_assert((BM / RS) % 2 == 0, "row pairs");
#pragma unroll 1
  for (int row = rr; row < BM; row += 2 * RS) {
    float4 v[2][kG2MaxSplit];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = m0 + row + h * RS;
      const bool ok = m < p.M && n < p.N;
      const float* src = p.kpart + (long)(ok ? m : 0) * p.N + (ok ? n : 0);
#pragma unroll
      for (int k = 0; k < kG2MaxSplit; ++k)
        v[h][k] = (ok && k < ks) ? *reinterpret_cast<const float4*>(src + k * slice) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 acc = v[h][0];
#pragma unroll
      for (int k = 1; k < kG2MaxSplit; ++k) {
        acc.x += v[h][k].x; acc.y += v[h][k].y; acc.z += v[h][k].z; acc.w += v[h][k].w;
      }
      bf16* d = reinterpret_cast<bf16*>(smem + (row + h * RS) * EPI_PITCH + c4 * 8);
      d[0] = (bf16)(acc.x + bv[0]);
      d[1] = (bf16)(acc.y + bv[1]);
      d[2] = (bf16)(acc.z + bv[2]);
      d[3] = (bf16)(acc.w + bv[3]);
    }
  }
  __syncthreads();
  g2_epilogue2<BM, BN, EPI_PITCH>(p, smem, m0, n0, tm, 0, p.cls_ory[0], p.cls_orx[0]);
}

// ---------------------------------------------------------------------------------------------
// gathered TN GEMM (weight gradient): dW[m][n] = sum_p dY[p][m] * Xcol[p][n],  n = (tap, c)
// ---------------------------------------------------------------------------------------------
template <int BM, int BN>
struct T2 {
  static constexpr int BK = 64;                       // pixels per K-step
  static constexpr int ACH = BM / 8, BCH = BN / 8;    // 16-B chunks per LDS row
  static constexpr int A_RPI = 64 / ACH, B_RPI = 64 / BCH;
  static constexpr int A_INS = BK / A_RPI / 4, B_INS = BK / B_RPI / 4;
  static constexpr int TM = BM / 32, TN = BN / 32;
  static constexpr int STAGE = BK * (BM + BN) * 2;
};

template <int RCH>
__device__ __forceinline__ int tr_swz(int row) {
  if constexpr (RCH >= 16) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  else if constexpr (RCH == 8) return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
  else return 0;
}

template <int BM, int BN, bool FAST>
__global__ void __launch_bounds__(256, 2) gemm_t2_kernel(T2Args p) {
  prefetch_kernargs<sizeof(T2Args)>();
  using T = T2<BM, BN>;
  constexpr int BK = T::BK;
  __shared__ __attribute__((aligned(16))) char smem[2 * T::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int lt = xcd_remap2(blockIdx.x, gridDim.x);
  const int split = lt / tiles, tt = lt % tiles;
  const int tm = tt / tiles_n, tn = tt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.P, kbeg + p.k_per_split);

  // opaque LDS DMA (common.h): keeps the next K-step's loads in flight across the tr reads
  const i32x4 rsA = raw_rsrc(p.dY, p.a_bytes);
  const i32x4 rsB = raw_rsrc(p.X, p.b_bytes);

  // A lanes: fixed column chunk (m), rows = pixels
  int a_row[T::A_INS];
  unsigned a_col[T::A_INS];
#pragma unroll
  for (int i = 0; i < T::A_INS; ++i) {
    const int row = (wid * T::A_INS + i) * T::A_RPI + lane / T::ACH;
    const int slot = lane % T::ACH;
    const int lch = slot ^ tr_swz<T::ACH>(row);
    a_row[i] = row;
    const int m = m0 + lch * 8;
    a_col[i] = m < p.M ? (unsigned)(m * 2) : kOOB;
  }
  // B lanes: fixed column chunk -> (tap dy/dx, channel) fixed over the K loop
  int b_row[T::B_INS], b_dy[T::B_INS], b_dx[T::B_INS];
  unsigned b_coff[T::B_INS];
  bool b_ok[T::B_INS];
#pragma unroll
  for (int i = 0; i < T::B_INS; ++i) {
    const int row = (wid * T::B_INS + i) * T::B_RPI + lane / T::BCH;
    const int slot = lane % T::BCH;
    const int lch = slot ^ tr_swz<T::BCH>(row);
    b_row[i] = row;
    const int n = n0 + lch * 8;
    const int t = n / p.Cs, c = n - t * p.Cs;
    b_ok[i] = n < p.N && t < p.ntaps;
    b_dy[i] = b_ok[i] ? p.tap_dy[t] : 0;
    b_dx[i] = b_ok[i] ? p.tap_dx[t] : 0;
    b_coff[i] = (unsigned)(c * 2);
  }
  const int ghw = p.GH * p.GW;
  const float inv_ghw = 1.f / (float)ghw, inv_gw = 1.f / (float)p.GW;
  // FAST pixel decomposition constants (see stage())
  int f_dimg[T::B_INS], f_dgy[T::B_INS];
  unsigned f_xoff[T::B_INS];
  bool f_xok[T::B_INS];
#pragma unroll
  for (int i = 0; i < T::B_INS; ++i) {
    const int r = b_row[i];
    int gx;
    if (ghw % 64 == 0) { f_dimg[i] = 0; f_dgy[i] = r / p.GW; gx = r % p.GW; }
    else { f_dimg[i] = r / ghw; const int rem = r % ghw; f_dgy[i] = rem / p.GW; gx = rem % p.GW; }
    const int sx = gx * p.SX + b_dx[i];
    f_xok[i] = b_ok[i] && sx >= 0 && sx < p.W;
    f_xoff[i] = (unsigned)(sx * p.Cs * 2) + b_coff[i];
  }

  auto stage = [&](int buf, int k0) {
    char* As = smem + buf * T::STAGE;
    char* Bs = As + BK * BM * 2;
#pragma unroll
    for (int i = 0; i < T::A_INS; ++i) {
      const int pix = k0 + a_row[i];
      const unsigned voff = (pix < kend && a_col[i] != kOOB) ? (unsigned)(pix * p.ldy * 2) + a_col[i] : kOOB;
      glds16_opaque(rsA, As + (wid * T::A_INS + i) * 1024, voff);
    }
    if constexpr (FAST) {
      // the 64 pixels of a K-step start at a multiple of 64 and tile whole image rows (or whole
      // images): per-lane (image, row, col) offsets are constants, only a scalar base moves
      const int img0 = k0 / ghw;
      const int gy0 = (k0 - img0 * ghw) / p.GW;
#pragma unroll
      for (int i = 0; i < T::B_INS; ++i) {
        const int pix = k0 + b_row[i];
        const int img = img0 + f_dimg[i];
        const int sy = (gy0 + f_dgy[i]) * p.SY + b_dy[i];
        const bool ok = f_xok[i] && pix < kend && sy >= 0 && sy < p.H;
        const unsigned voff = ok ? (unsigned)((((long)img * p.H + sy) * p.W) * p.Cs * 2) + f_xoff[i] : kOOB;
        glds16_opaque(rsB, Bs + (wid * T::B_INS + i) * 1024, voff);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < T::B_INS; ++i) {
      const int pix = k0 + b_row[i];
      // pix -> (img, gy, gx) with a float reciprocal + exact integer correction
      int img = (int)((float)pix * inv_ghw);
      int rem = pix - img * ghw;
      if (rem < 0) { img--; rem += ghw; } else if (rem >= ghw) { img++; rem -= ghw; }
      int gy = (int)((float)rem * inv_gw);
      int gx = rem - gy * p.GW;
      if (gx < 0) { gy--; gx += p.GW; } else if (gx >= p.GW) { gy++; gx -= p.GW; }
      const int sy = gy * p.SY + b_dy[i], sx = gx * p.SX + b_dx[i];
      const bool ok = b_ok[i] && pix < kend && sy >= 0 && sy < p.H && sx >= 0 && sx < p.W;
      const unsigned voff = ok ? (unsigned)((((long)img * p.H + sy) * p.W + sx) * p.Cs * 2) + b_coff[i] : kOOB;
      glds16_opaque(rsB, Bs + (wid * T::B_INS + i) * 1024, voff);
    }
  };
  auto tr_read = [&](const char* base, int rowbytes, int krow, int col0, auto rch) -> bf16x4 {
    constexpr int RCH = decltype(rch)::value;
    const int i = lane & 15, q = i >> 2, pp = i & 3;
    const int row = krow + q;
    const int col = col0 + 4 * pp;
    const int chn = col >> 3, within = (col & 7) * 2;
    const char* addr = base + row * rowbytes + ((chn ^ tr_swz<RCH>(row)) << 4) + within;
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(const_cast<char*>(addr)));
  };

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = p.bias_slab != nullptr && tn == 0;
  float bias_acc = 0.f;

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) stage(0, kbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(cur ^ 1, kbeg + (kt + 1) * BK);
    const char* As = smem + cur * T::STAGE;
    const char* Bs = As + BK * BM * 2;
    if (do_bias) {
      constexpr int RS = 256 / BM;
      const int col = tid % BM, rr = tid / BM;
      const int chn = col >> 3, w = (col & 7) * 2;
      for (int r = rr; r < BK; r += RS)
        bias_acc += (float)*reinterpret_cast<const bf16*>(As + r * BM * 2 + ((chn ^ tr_swz<T::ACH>(r)) << 4) + w);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int krow = kk * 32 + 8 * (lane >> 4);
      bf16x8 a[T::TM], b[T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i) {
        const bf16x4 lo = tr_read(As, BM * 2, krow, wm * (BM / 2) + i * 16, std::integral_constant<int, T::ACH>{});
        const bf16x4 hi = tr_read(As, BM * 2, krow + 4, wm * (BM / 2) + i * 16, std::integral_constant<int, T::ACH>{});
        a[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < T::TN; ++j) {
        const bf16x4 lo = tr_read(Bs, BN * 2, krow, wn * (BN / 2) + j * 16, std::integral_constant<int, T::BCH>{});
        const bf16x4 hi = tr_read(Bs, BN * 2, krow + 4, wn * (BN / 2) + j * 16, std::integral_constant<int, T::BCH>{});
        b[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }

  float* out = p.slab + (long)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (m < p.M && n < p.N) out[(long)m * p.N + n] = acc[i][j][r];
      }
    }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);
    constexpr int RS = 256 / BM;
    __syncthreads();
    red[tid] = bias_acc;
    __syncthreads();
    if (tid < BM) {
      float s = 0.f;
      for (int k = 0; k < RS; ++k) s += red[tid + k * BM];
      if (m0 + tid < p.M) p.bias_slab[(long)split * p.M + m0 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
// LDS ring depth: 3 stages wherever the deeper ring still leaves two workgroups per CU (every
// tile but 128x128), else 2 (g2_stages() == 0: that rule)
static int g2_stages() {
  static const int v = [] {
    const char* e = std::getenv("DCNN_G2_STAGES");  // experiment hook: force 2 or 3 ring stages
    return e ? std::atoi(e) : 0;
  }();
  return v == 2 || v == 3 ? v : 0;
}

// split-K partial workspace per (device, stream): grow-only, allocated in the eager warm-up
// before a graph captures the step. An outgrown buffer is kept (a graph captured earlier still
// reads it). A capture whose stream has no large-enough workspace yet (warm-up ran on another
// stream, e.g. torch.cuda.graph's side stream) borrows the largest one of the device: its owner is
// the warm-up stream, which the graph's replays are ordered with; with none large enough it throws.
static float* g2_kpart(size_t bytes, hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<float*, size_t>> ws;
  static std::vector<float*> retired;  // (never freed: captured graphs may hold them)
  int dev = 0;
  DCNN_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto& e = ws[{dev, s}];
  if (e.second < bytes) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    DCNN_HIP_CHECK(hipStreamIsCapturing(s, &st));
    if (st != hipStreamCaptureStatusNone) {
      const std::pair<float*, size_t>* best = nullptr;
      for (const auto& kv : ws)
        if (kv.first.first == dev && kv.second.second >= bytes && (!best || kv.second.second > best->second))
          best = &kv.second;
      if (best) return best->first;
      throw std::runtime_error("gemm_g2: split-K workspace must grow outside graph capture (run a step eagerly first)");
    }
    if (e.first) retired.push_back(e.first);
    const size_t n = bytes > (size_t)(32 << 20) ? bytes : (size_t)(32 << 20);
    DCNN_HIP_CHECK(hipMalloc(&e.first, n));
    e.second = n;
  }
  return e.first;
}

// tuning / test hook: split-K for long-K 1x1 GEMMs on small grids (DCNN_G2_SPLITK=0: off)
static int g_g2_splitk = [] {
  const char* v = std::getenv("DCNN_G2_SPLITK");
  return (v && v[0] == '0') ? 0 : 1;
}();
void gemm_g2_set_splitk(int on) { g_g2_splitk = on; }
int gemm_g2_splitk_enabled() { return g_g2_splitk; }

// K slices of a plain 1x1 GEMM (one tap, unit strides, no row classes) with K >= 1024 whose tile
// grid cannot fill the chip: enough slices for ~512 workgroups, each keeping >= 4 K-steps
static int g2_ksplit(const G2Args& a, int tiles, int bk) {
  if (g_g2_splitk != 1 || a.ntaps != 1 || a.ncls > 1 || a.Cs < 1024 || tiles >= 256) return 1;
  if (a.tap_dy[0] != 0 || a.tap_dx[0] != 0 || a.SY != 1 || a.SX != 1 || a.OSY != 1 || a.OSX != 1 ||
      a.GH != a.H || a.GW != a.W || a.OH != a.GH || a.OW != a.GW || a.ldc != a.N)
    return 1;
  const int nk = (a.Cs + bk - 1) / bk;
  int ks = (512 + tiles - 1) / tiles;
  if (ks > nk / 4) ks = nk / 4;
  if (ks > kG2MaxSplit) ks = kG2MaxSplit;
  return ks < 2 ? 1 : ks;
}

template <int BM, int BN, int BK, bool UNI>
static void launch_g2(const G2Args& a0, hipStream_t s) {
  const int tiles = ((a0.M + BM - 1) / BM) * ((a0.N + BN - 1) / BN);
  G2Args a = a0;
  a.ksplit = 1;
  if constexpr (BK == 64 && UNI) {  // (split-K shapes: K >= 1024, so always 64-wide uniform K-steps)
    a.ksplit = g2_ksplit(a0, tiles, BK);
    if (a.ksplit > 1) {
      a.kpart = g2_kpart((size_t)a.ksplit * a.M * a.N * 4, s);
      hipLaunchKernelGGL((gemm_g2_kernel<BM, BN, BK, UNI, 2, true>), dim3(tiles * a.ksplit), dim3(256), 0, s, a);
      DCNN_LAUNCH_CHECK();
      a.zero_ptr = nullptr;  // (zeroed by the GEMM launch)
      hipLaunchKernelGGL((g2_splitk_epi_kernel<BM, BN>), dim3(tiles), dim3(256), 0, s, a);
      DCNN_LAUNCH_CHECK();
      return;
    }
  }
  // single-step K loops (1x1 convs on 32-64 channels and their data gradients) never use a third
  // ring stage: 2 stages there free LDS for one more resident workgroup per CU (layer-1 1x1 dgrad
  // 27.0 -> 22.3 us; two-step loops keep 3 stages: both steps in flight from the prologue)
  int ksteps = 0;
  for (int c = 0; c < a.ncls; ++c) {
    const int k = a.cls_nt[c] * ((a.Cs + BK - 1) / BK);
    ksteps = k > ksteps ? k : ksteps;
  }
  // The 128 x 64 tile also stays at 2 stages: there the third stage costs an occupancy step (3 -> 2
  // workgroups per CU: 131 VGPRs, 49 vs 74 KB of LDS) that the deeper ring does not buy back.
  // ResNet-18 b256 step, per-kernel trace (tools/gpu/g2stages_prof.sh): the l2.b1c1 data gradient
  // 75.6 -> 67.1 us and the l2.proj one 29.3 -> 24.8 us at 2 stages, while the 64 x 128 / 64 x 64
  // tiles (2 -> 3 and 3 -> 5 per CU at 2 stages) got slower there (26.8 -> 30.0, 28.8 -> 37.6 us).
  constexpr bool deep = !(BM == 128 && BN == 64);
  const int stages = g2_stages() ? g2_stages()
                                 : ((deep && 2 * G2<BM, BN, BK, UNI, 3>::LDS <= 163840 && ksteps > 1) ? 3 : 2);
  if (stages == 3)
    hipLaunchKernelGGL((gemm_g2_kernel<BM, BN, BK, UNI, 3>), dim3(tiles), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_g2_kernel<BM, BN, BK, UNI, 2>), dim3(tiles), dim3(256), 0, s, a);
  DCNN_LAUNCH_CHECK();
}

// Tile choice: the largest tile that still gives >= ~2 workgroups per CU.
void g2_tile(int M, int N, int* bm, int* bn) {
  static const int force = [] {  // experiment hook: DCNN_G2_TILE=BMxBN forces one tile shape
    const char* e = std::getenv("DCNN_G2_TILE");
    int m = 0, n = 0;
    return (e && std::sscanf(e, "%dx%d", &m, &n) == 2) ? m * 1000 + n : 0;
  }();
  if (force) { *bm = force / 1000; *bn = force % 1000; return; }
  auto tiles = [&](int m, int n) { return (long)((M + m - 1) / m) * ((N + n - 1) / n); };
  // (DCNN_G2_SPLITK=2 experiment: grids below 192 tiles of 64 x 64 on 32 x 64 tiles instead)
  if (g_g2_splitk == 2 && N <= 256 && tiles(64, 64) < 192) { *bm = 32; *bn = 64; return; }
  if (N >= 128 && tiles(128, 128) >= 480) { *bm = 128; *bn = 128; return; }
  // wide-N, mid-M (8x8-map convs of 256 channels, M = 16384): 64 x 128 beats 128 x 64 at the
  // same tile count (layer-3 strided forward 32.7 -> 29.5 us, layer-4 strided dgrad 42.7 -> 40.0)
  if (N >= 128 && tiles(64, 128) >= 480 && tiles(128, 64) < 640) { *bm = 64; *bn = 128; return; }
  if (tiles(128, 64) >= 480 || N < 128) {
    *bm = tiles(128, 64) >= 400 ? 128 : 64;
    *bn = 64;
    return;
  }
  if (tiles(64, 128) >= 400) { *bm = 64; *bn = 128; return; }
  *bm = 64;
  *bn = 64;
}

int gemm_g2_stat_rows(int M, int N) {
  int bm, bn;
  g2_tile(M, N, &bm, &bn);
  return (M + bm - 1) / bm;
}

int gemm_g2_row_tile(int M, int N) {
  int bm, bn;
  g2_tile(M, N, &bm, &bn);
  return bm;
}

void gemm_g2(const G2Args& a_in, hipStream_t s) {
  G2Args a = a_in;
  if (a.N % 8 != 0 || a.Cs % 8 != 0 || a.ldb % 8 != 0 || a.ldc % 8 != 0 || a.ntaps > 64 || a.ntaps < 1)
    throw std::runtime_error("gemm_g2: unsupported shape (needs N, Cs, ldb, ldc multiples of 8, 1..64 taps)");
  int bm, bn;
  g2_tile(a.M, a.N, &bm, &bn);
  if (a.ncls <= 1) {
    a.ncls = 1; a.cls_rows = a.M;
    a.cls_t0[0] = 0; a.cls_nt[0] = a.ntaps; a.cls_ory[0] = a.ORY; a.cls_orx[0] = a.ORX;
  } else {
    if (a.ncls > 4 || a.cls_rows <= 0 || a.cls_rows % bm || a.ncls * a.cls_rows != a.M)
      throw std::runtime_error("gemm_g2: grouped classes need <= 4 classes of equal rows, a multiple of the row tile");
    for (int c = 0; c < a.ncls; ++c)
      if (a.cls_nt[c] < 0 || a.cls_t0[c] < 0 || a.cls_t0[c] + a.cls_nt[c] > a.ntaps)
        throw std::runtime_error("gemm_g2: class tap range out of bounds");
  }
  {
    const FastDiv f1 = make_fastdiv((unsigned)(a.GH * a.GW)), f2 = make_fastdiv((unsigned)a.GW);
    a.fd_ghw[0] = f1.mul; a.fd_ghw[1] = f1.shr; a.fd_ghw[2] = f1.d;
    a.fd_gw[0] = f2.mul; a.fd_gw[1] = f2.shr; a.fd_gw[2] = f2.d;
    if ((long)a.M >= (1l << 31)) throw std::runtime_error("gemm_g2: M >= 2^31");
  }
  const int bk = (a.Cs % 64 == 0) ? 64 : 32;
  const bool uni = a.Cs % bk == 0;
#define DCNN_G2(BM, BN, BK, U) if (bm == BM && bn == BN && bk == BK && uni == U) return launch_g2<BM, BN, BK, U>(a, s)
  DCNN_G2(128, 128, 64, true);
  DCNN_G2(128, 64, 64, true);
  DCNN_G2(64, 128, 64, true);
  DCNN_G2(64, 64, 64, true);
  DCNN_G2(32, 64, 64, true);
  DCNN_G2(128, 128, 32, true);
  DCNN_G2(128, 64, 32, true);
  DCNN_G2(64, 128, 32, true);
  DCNN_G2(64, 64, 32, true);
  DCNN_G2(128, 128, 32, false);
  DCNN_G2(128, 64, 32, false);
  DCNN_G2(64, 128, 32, false);
  DCNN_G2(64, 64, 32, false);
#undef DCNN_G2
  throw std::runtime_error("gemm_g2: no variant");
}

template <int BM, int BN, bool FAST>
static void launch_t2(T2Args a, int splits, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_t2_kernel<BM, BN, FAST>), dim3(tiles * splits), dim3(256), 0, s, a);
  DCNN_LAUNCH_CHECK();
}

void t2_tile(int M, int N, int* bm, int* bn) {
  // 128 x 64 once M >= 128: twice the tiles of 128 x 128, so half the split-K slices and slab
  // traffic (strided 3x3 weight gradients of layers 2-4: 43 / 39 / 38 -> 33 / 33 / 32 us at
  // batch 256); 128-wide N tiles only when M is a single 64-row tile
  *bm = M >= 128 ? 128 : 64;
  *bn = (N >= 128 && M < 128) ? 128 : 64;
}

static int g_t2_target = 512;  // split-K target workgroups of the gathered weight gradient
void gemm_t2_set_split_target(int t) { g_t2_target = t < 1 ? 1 : t; }

int gemm_t2_splits(int M, int N, int P) {
  int bm, bn;
  t2_tile(M, N, &bm, &bn);
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  long splits = (g_t2_target + tiles - 1) / tiles;
  // at least 256 reduction pixels per split (1024: ResNet-50 b32 7.9k -> 7.2k img/s,
  // profiles/wgrad_splits_r3.md)
  constexpr long min_k = 256;
  const long max_by_k = P / min_k > 0 ? P / min_k : 1;
  if (splits > max_by_k) splits = max_by_k;
  const long max_by_mem = (48l << 20) / (4l * M * N) > 0 ? (48l << 20) / (4l * M * N) : 1;
  if (splits > max_by_mem) splits = max_by_mem;
  if (splits < 1) splits = 1;
  if (splits > 256) splits = 256;
  return (int)splits;
}

void gemm_t2(T2Args a, int splits, hipStream_t s) {
  if (a.M % 8 != 0 || a.N % 8 != 0 || a.Cs % 8 != 0 || a.ldy % 8 != 0 || a.ntaps > 64)
    throw std::runtime_error("gemm_t2: unsupported shape");
  int bm, bn;
  t2_tile(a.M, a.N, &bm, &bn);
  const int per = (a.P + splits - 1) / splits;
  a.k_per_split = ((per + 63) / 64) * 64;
  const int ghw = a.GH * a.GW;
  const bool fast = (ghw % 64 == 0 && 64 % a.GW == 0) || (64 % ghw == 0);
#define DCNN_T2(BM, BN) \
  if (bm == BM && bn == BN) return fast ? launch_t2<BM, BN, true>(a, splits, s) : launch_t2<BM, BN, false>(a, splits, s)
  DCNN_T2(128, 128);
  DCNN_T2(128, 64);
  DCNN_T2(64, 128);
  DCNN_T2(64, 64);
#undef DCNN_T2
  throw std::runtime_error("gemm_t2: no variant");
}

}  // namespace dcnn
