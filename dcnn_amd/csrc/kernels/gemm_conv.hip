// Implicit-GEMM convolution and dense GEMM on CDNA4 MFMA (gfx950), bf16 in / fp32 accumulate.
//
// Replaces the reference's im2col + cuBLAS SGEMM + NCHW<->CNHW transposes + bias kernels
// (src/nn/layers_impl/cuda/conv2d_ops.cu:18-128, src/tensor/cuda/tensor_kernels.cu:17-135,
//  src/ops/cuda/kernels.cu:245 nchw_cnhw_transpose_tiled, src/math/cuda/gemm.cu:28) with:
//
//   * gemm_nt  : C[M][N] = A[M][K] . B[N][K]^T, both operands K-contiguous.
//                A is gathered on the fly from an NHWC activation (conv forward: output pixel x
//                tap x Cin; conv dgrad: input pixel x tap x Cout with stride-aware validity),
//                or is a plain row-major matrix (dense).  B = weights [Cout][KH][KW][Cin]
//                (forward) or the transposed copy [Cin][KH][KW][Cout] (dgrad).
//                Fused epilogue: bias, residual add, ReLU, bf16/fp32 store, and per-channel
//                (sum, sum^2) partials for a following BatchNorm (saves one full HBM read).
//   * gemm_tn  : weight gradient dW[Cout][KH*KW*Cin] = sum_p dY[p][Cout] x X(p, tap, ci)
//                (both operands K(=pixel)-major, read from LDS with ds_read_b64_tr_b16),
//                split-K over pixels into fp32 slabs + a reduce kernel that accumulates
//                (beta = 1) into the fp32 master gradient; conv/dense bias gradients are
//                column sums of the dY tiles already staged in LDS.
//
// Tiles are wave64-native: 4 waves (2x2) per 256-thread workgroup, each wave a
// (BM/2)x(BN/2) block of 16x16x32 MFMAs; LDS 16-byte chunks are XOR-swizzled so the
// fragment reads are bank-conflict free; global->LDS staging is register-pipelined (tile k+1
// loads in flight while tile k is multiplied, one barrier per K-step); the block index is
// remapped so that each XCD (private L2) works on a contiguous range of output tiles.
#include <algorithm>

#include "common.h"
#include "api.h"

namespace dcnn {

enum GatherMode { kPlain = 0, kConvFwd = 1, kConvDgrad = 2 };



__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // Bijective: block b and b+8 share an XCD (round-robin dispatch); give every XCD a
  // contiguous run of logical tile ids so neighbouring tiles share that XCD's L2.
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ----------------------------------------------------------------------------------------
// gemm_nt
// ----------------------------------------------------------------------------------------
template <int BM, int BN, int BK, bool VEC>
struct NtTile {
  static constexpr int CPR = BK / 8;                 // 16-byte chunks per LDS row
  static constexpr int RPB = 256 / (BK * 2);         // LDS rows per 256-byte bank row
  static constexpr int A_CH = BM * CPR / 256;        // A chunks per thread per K-step
  static constexpr int B_CH = BN * CPR / 256;
  static constexpr int TM = BM / 32, TN = BN / 32;   // 16x16 subtiles per wave
  static constexpr int LDS_BYTES = 2 * (BM + BN) * BK * 2;
  __device__ static __forceinline__ int off(int row, int ch) {
    return row * (BK * 2) + ((ch ^ ((row / RPB) % CPR)) << 4);
  }
};

template <int BM, int BN, int BK, bool VEC>
__global__ void __launch_bounds__(256, 2) gemm_nt_kernel(NtArgs p) {
  using T = NtTile<BM, BN, BK, VEC>;
  __shared__ __attribute__((aligned(16))) char smem[T::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int lt = xcd_remap(blockIdx.x, nwg);
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // Per-thread A rows (fixed over K): decompose GEMM row -> (image, y, x).
  int a_row[T::A_CH], a_img[T::A_CH], a_y[T::A_CH], a_x[T::A_CH];
  bool a_ok[T::A_CH];
  const int ch_t = tid % T::CPR;
#pragma unroll
  for (int i = 0; i < T::A_CH; ++i) {
    const int r = tid / T::CPR + i * (256 / T::CPR);
    const int m = m0 + r;
    a_row[i] = r;
    a_ok[i] = m < p.M;
    const int hw = p.gh * p.gw;
    const int mm = a_ok[i] ? m : 0;
    a_img[i] = mm / hw;
    const int rem = mm - a_img[i] * hw;
    a_y[i] = rem / p.gw;
    a_x[i] = rem - a_y[i] * p.gw;
  }

  uint4 ra[T::A_CH], rb[T::B_CH];

  auto load_tile = [&](int k0) {
    // ---- A ----
    if constexpr (VEC) {
      int tap = 0, c0 = k0, ky = 0, kx = 0;
      if (p.mode != kPlain) {
        tap = k0 / p.cs;
        c0 = k0 - tap * p.cs;
        ky = tap / p.kw;
        kx = tap - ky * p.kw;
      }
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        bool ok = a_ok[i];
        long addr;
        if (p.mode == kPlain) {
          addr = (long)(m0 + a_row[i]) * p.lda + k0 + ch_t * 8;
          ok = ok && (k0 + ch_t * 8 < p.K);
        } else {
          int sy, sx;
          if (p.mode == kConvFwd) {
            sy = a_y[i] * p.strh - p.padh + ky;
            sx = a_x[i] * p.strw - p.padw + kx;
          } else {
            const int ty = a_y[i] + p.padh - ky, tx = a_x[i] + p.padw - kx;
            const bool dv = ty >= 0 && tx >= 0 && (ty % p.strh) == 0 && (tx % p.strw) == 0;
            sy = dv ? ty / p.strh : -1;
            sx = dv ? tx / p.strw : -1;
          }
          ok = ok && sy >= 0 && sy < p.sh && sx >= 0 && sx < p.sw;
          addr = (((long)a_img[i] * p.sh + sy) * p.sw + sx) * p.cs + c0 + ch_t * 8;
        }
        ra[i] = ok ? *reinterpret_cast<const uint4*>(p.A + addr) : make_uint4(0, 0, 0, 0);
      }
    } else {
      // Generic element-wise gather (odd Cin such as the RGB stem, or K % 8 != 0).
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        bf16 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + ch_t * 8 + e;
          bool ok = a_ok[i] && k < p.K;
          float val = 0.f;
          if (ok) {
            if (p.mode == kPlain) {
              val = (float)p.A[(long)(m0 + a_row[i]) * p.lda + k];
            } else {
              const int tap = k / p.cs, c = k - tap * p.cs;
              const int ky = tap / p.kw, kx = tap - ky * p.kw;
              int sy, sx;
              if (p.mode == kConvFwd) {
                sy = a_y[i] * p.strh - p.padh + ky;
                sx = a_x[i] * p.strw - p.padw + kx;
              } else {
                const int ty = a_y[i] + p.padh - ky, tx = a_x[i] + p.padw - kx;
                const bool dv = ty >= 0 && tx >= 0 && (ty % p.strh) == 0 && (tx % p.strw) == 0;
                sy = dv ? ty / p.strh : -1;
                sx = dv ? tx / p.strw : -1;
              }
              if (sy >= 0 && sy < p.sh && sx >= 0 && sx < p.sw)
                val = (float)p.A[(((long)a_img[i] * p.sh + sy) * p.sw + sx) * p.cs + c];
            }
          }
          v[e] = (bf16)val;
        }
        ra[i] = *reinterpret_cast<uint4*>(v);
      }
    }
    // ---- B (weights, row n, K contiguous) ----
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i) {
      const int r = tid / T::CPR + i * (256 / T::CPR);
      const int n = n0 + r;
      const int k = k0 + ch_t * 8;
      if constexpr (VEC) {
        const bool ok = n < p.N && k < p.K;
        rb[i] = ok ? *reinterpret_cast<const uint4*>(p.B + (long)n * p.ldb + k) : make_uint4(0, 0, 0, 0);
      } else {
        bf16 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (n < p.N && k + e < p.K) ? p.B[(long)n * p.ldb + k + e] : (bf16)0.f;
        rb[i] = *reinterpret_cast<uint4*>(v);
      }
    }
  };

  auto store_tile = [&](int buf) {
    char* As = smem + buf * (BM + BN) * BK * 2;
    char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) *reinterpret_cast<uint4*>(As + T::off(a_row[i], ch_t)) = ra[i];
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i) {
      const int r = tid / T::CPR + i * (256 / T::CPR);
      *reinterpret_cast<uint4*>(Bs + T::off(r, ch_t)) = rb[i];
    }
  };

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    const char* As = smem + cur * (BM + BN) * BK * 2;
    const char* Bs = As + BM * BK * 2;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 a[T::TM], b[T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(As + T::off(wm * (BM / 2) + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + T::off(wn * (BN / 2) + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue ----
  // BatchNorm statistics about a per-(M-wave, column) pivot, merged with Chan's update (no
  // cancellation, fixed order)
  float csum[T::TN], csq[T::TN], ccnt[T::TN], cpiv[T::TN];
#pragma unroll
  for (int j = 0; j < T::TN; ++j) csum[j] = csq[j] = ccnt[j] = 0.f;
#pragma unroll
  for (int j = 0; j < T::TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
    const bool nok = n < p.N;
    const float bv = (p.bias && nok) ? p.bias[n] : 0.f;
    cpiv[j] = __shfl(p.out_f32 ? acc[0][j][0] + bv : (float)(bf16)(acc[0][j][0] + bv), lane & 15, 64);
#pragma unroll
    for (int i = 0; i < T::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (nok && m < p.M) {
          float v = acc[i][j][r] + bv;
          const long o = (long)m * p.ldc + n;
          if (p.residual) v += (float)p.residual[o];
          if (p.relu) v = fmaxf(v, 0.f);
          if (p.out_f32) {
            reinterpret_cast<float*>(p.C)[o] = v;
          } else {
            const bf16 h = (bf16)v;
            reinterpret_cast<bf16*>(p.C)[o] = h;
            v = (float)h;  // statistics of the stored values
          }
          const float d = v - cpiv[j];
          csum[j] += d;
          csq[j] += d * d;
          ccnt[j] += 1.f;
        }
      }
    }
  }
  if (p.stats) {
    // reduce over the 4 lane-rows groups of the wave, then over the 2 waves along M
    float* red = reinterpret_cast<float*>(smem);  // reuse LDS (loop finished, barrier passed)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) {
      float s = csum[j], q = csq[j], c = ccnt[j];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      c += __shfl_xor(c, 16, 64);
      c += __shfl_xor(c, 32, 64);
      if (lane < 16) {
        const int col = wn * (BN / 2) + j * 16 + lane;
        red[(wm * 4 + 0) * BN + col] = s;
        red[(wm * 4 + 1) * BN + col] = q;
        red[(wm * 4 + 2) * BN + col] = cpiv[j];
        red[(wm * 4 + 3) * BN + col] = c;
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      const int n = n0 + c;
      if (n < p.N) {
        Welford t = welford_from_shifted(red[3 * BN + c], red[2 * BN + c], red[0 * BN + c], red[1 * BN + c]);
        t = welford_merge(t, welford_from_shifted(red[7 * BN + c], red[6 * BN + c], red[4 * BN + c], red[5 * BN + c]));
        store_welford(p.stats, tm, p.N, n, t);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// gemm_tn (weight gradients), split-K over the pixel dimension
// ----------------------------------------------------------------------------------------


template <int ROWCH>
__device__ __forceinline__ int tn_swz(int row) {
  if constexpr (ROWCH >= 16) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  else if constexpr (ROWCH == 8) return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
  else return 0;
}

template <int BM, int BN, int BK, bool VEC>
__global__ void __launch_bounds__(256, 2) gemm_tn_kernel(TnArgs p) {
  constexpr int ACH = BM / 8, BCH = BN / 8;            // chunks per LDS row
  constexpr int A_CH = BK * ACH / 256, B_CH = BK * BCH / 256;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int lt = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lt / tiles, tt = lt % tiles;
  const int tm = tt / tiles_n, tn = tt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.P, kbeg + p.k_per_split);

  // column tap (fixed for the tile in the vector conv path: the BN channels lie in one tap)
  int tap_y = 0, tap_x = 0, c0 = n0;
  if (p.mode == kConvFwd && VEC) {
    const int tap = n0 / p.cs;
    c0 = n0 - tap * p.cs;
    tap_y = tap / p.kw;
    tap_x = tap - tap_y * p.kw;
  }
  const bool do_bias = p.bias_slab != nullptr && tn == 0;
  float bias_acc = 0.f;

  uint4 ra[A_CH], rb[B_CH];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int id = tid + i * 256, r = id / ACH, c = id % ACH;
      const int pix = k0 + r, m = m0 + c * 8;
      if constexpr (VEC) {
        const bool ok = pix < kend && m < p.M;
        ra[i] = ok ? *reinterpret_cast<const uint4*>(p.dY + (long)pix * p.M + m) : make_uint4(0, 0, 0, 0);
      } else {
        bf16 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = (pix < kend && m + e < p.M) ? p.dY[(long)pix * p.M + m + e] : (bf16)0.f;
        ra[i] = *reinterpret_cast<uint4*>(v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int id = tid + i * 256, r = id / BCH, c = id % BCH;
      const int pix = k0 + r, n = n0 + c * 8;
      const bool pok = pix < kend;
      int img = 0, y = 0, x = 0;
      if (p.mode == kConvFwd) {
        const int hw = p.gh * p.gw;
        const int pp = pok ? pix : 0;
        img = pp / hw;
        const int rem = pp - img * hw;
        y = rem / p.gw;
        x = rem - y * p.gw;
      }
      if constexpr (VEC) {
        bool ok = pok && n < p.N;
        long addr;
        if (p.mode == kPlain) {
          addr = (long)pix * p.ldx + n;
        } else {
          const int sy = y * p.strh - p.padh + tap_y, sx = x * p.strw - p.padw + tap_x;
          ok = ok && sy >= 0 && sy < p.sh && sx >= 0 && sx < p.sw;
          addr = (((long)img * p.sh + sy) * p.sw + sx) * p.cs + c0 + c * 8;
        }
        rb[i] = ok ? *reinterpret_cast<const uint4*>(p.X + addr) : make_uint4(0, 0, 0, 0);
      } else {
        bf16 v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int nn = n + e;
          float val = 0.f;
          if (pok && nn < p.N) {
            if (p.mode == kPlain) {
              val = (float)p.X[(long)pix * p.ldx + nn];
            } else {
              const int tap = nn / p.cs, cc = nn - tap * p.cs;
              const int ky = tap / p.kw, kx = tap - ky * p.kw;
              const int sy = y * p.strh - p.padh + ky, sx = x * p.strw - p.padw + kx;
              if (sy >= 0 && sy < p.sh && sx >= 0 && sx < p.sw)
                val = (float)p.X[(((long)img * p.sh + sy) * p.sw + sx) * p.cs + cc];
            }
          }
          v[e] = (bf16)val;
        }
        rb[i] = *reinterpret_cast<uint4*>(v);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int id = tid + i * 256, r = id / ACH, c = id % ACH;
      *reinterpret_cast<uint4*>(As + r * BM * 2 + ((c ^ tn_swz<ACH>(r)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int id = tid + i * 256, r = id / BCH, c = id % BCH;
      *reinterpret_cast<uint4*>(Bs + r * BN * 2 + ((c ^ tn_swz<BCH>(r)) << 4)) = rb[i];
    }
  };
  // transposed fragment read: lane gets rows k..k+3 of column (col0 + lane&15)
  auto tr_read = [&](const char* base, int rowch, int rowbytes, int krow, int col0) -> bf16x4 {
    const int i = lane & 15, q = i >> 2, pp = i & 3;
    const int row = krow + q;
    const int col = col0 + 4 * pp;             // element column
    const int ch = col >> 3, within = (col & 7) * 2;
    int swz;
    if (rowch >= 16) swz = ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
    else if (rowch == 8) swz = (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
    else swz = 0;
    const char* addr = base + row * rowbytes + ((ch ^ swz) << 4) + within;
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(const_cast<char*>(addr)));
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile(kbeg);
    store_tile(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile(kbeg + (kt + 1) * BK);
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
    if (do_bias) {
      // column sums of the staged dY tile (conv / dense bias gradient)
      constexpr int RSTEP = 256 / BM > 0 ? 256 / BM : 1;
      const int col = tid % BM, r0 = tid / BM;
      if (tid < BM * RSTEP) {
        const int ch = col >> 3, w = (col & 7) * 2;
        for (int r = r0; r < BK; r += RSTEP)
          bias_acc += (float)*reinterpret_cast<const bf16*>(As + r * BM * 2 + ((ch ^ tn_swz<ACH>(r)) << 4) + w);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int krow = kk * 32 + 8 * (lane >> 4);
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x4 lo = tr_read(As, ACH, BM * 2, krow, wm * (BM / 2) + i * 16);
        const bf16x4 hi = tr_read(As, ACH, BM * 2, krow + 4, wm * (BM / 2) + i * 16);
        a[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bf16x4 lo = tr_read(Bs, BCH, BN * 2, krow, wn * (BN / 2) + j * 16);
        const bf16x4 hi = tr_read(Bs, BCH, BN * 2, krow + 4, wn * (BN / 2) + j * 16);
        b[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  float* out = p.slab + (long)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (m < p.M && n < p.N) out[(long)m * p.N + n] = acc[i][j][r];
      }
    }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);
    constexpr int RSTEP = 256 / BM > 0 ? 256 / BM : 1;
    __syncthreads();
    red[tid] = (tid < BM * RSTEP) ? bias_acc : 0.f;
    __syncthreads();
    if (tid < BM) {
      float s = 0.f;
      for (int k = 0; k < RSTEP; ++k) s += red[tid + k * BM];
      if (m0 + tid < p.M) p.bias_slab[(long)split * p.M + m0 + tid] = s;
    }
  }
}

// out[i] (+)= sum_s slab[s][i]. 2-D grid: blockIdx.y picks a group of splits so the reduce has
// enough workgroups to fill the chip even when the output (a weight gradient) is tiny; groups
// combine with float atomics (accumulate semantics, the gradient buffer is zeroed per step).
// One launch reduces up to two slabs (a weight gradient and its bias gradient): blocks
// [0, gxa) take segment a, the rest segment b — one kernel boundary per layer instead of two.
struct SplitkSeg {
  const float* slab;
  float* out;
  long n;
};

__device__ __forceinline__ void splitk_segment(const SplitkSeg g, long bid, long nblk, int splits, int accumulate) {
  const long n = g.n, n4 = n / 4;
  const float* __restrict__ slab = g.slab;
  float* __restrict__ out = g.out;
  for (long i = bid * blockDim.x + threadIdx.x; i < n4; i += nblk * blockDim.x) {
    // 8 independent 16-byte loads in flight per lane: the slab stream is latency-bound otherwise
    float4 s = make_float4(0, 0, 0, 0);
    int k = 0;
    for (; k + 8 <= splits; k += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4*>(slab + (long)(k + u) * n)[i];
#pragma unroll
      for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; k < splits; ++k) {
      const float4 v = reinterpret_cast<const float4*>(slab + (long)k * n)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (accumulate) {
      float4 c = reinterpret_cast<float4*>(out)[i];
      c.x += s.x; c.y += s.y; c.z += s.z; c.w += s.w;
      reinterpret_cast<float4*>(out)[i] = c;
    } else {
      reinterpret_cast<float4*>(out)[i] = s;
    }
  }
  for (long i = n4 * 4 + bid * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += slab[(long)k * n + i];
    out[i] = accumulate ? out[i] + s : s;
  }
}

// Split-K combine: every output element is summed by ONE thread over the splits in index order
// (deterministic, no float atomics); up to two slabs (a weight gradient and its bias gradient)
// per launch: blocks [0, gxa) take segment a, the rest segment b.
__global__ void splitk_reduce_kernel(SplitkSeg a, SplitkSeg b, int gxa, int splits, int accumulate) {
  if ((int)blockIdx.x < gxa)
    splitk_segment(a, blockIdx.x, gxa, splits, accumulate);
  else
    splitk_segment(b, blockIdx.x - gxa, gridDim.x - gxa, splits, accumulate);
}

// Deferred split-K reduction: the fp32 slabs of many weight gradients summed into their
// gradients in ONE launch (api.h MultiRed). A work unit is (entry, 4 / wpc chunks of 256 floats):
// each chunk gets wpc waves (1, 2 or 4 by split count, so few-split slabs do not leave waves
// idle), wave j of a chunk sums splits {G wpc g + G j .. + G - 1} for every group g in order with
// all G loads of a group in flight, the chunk's waves meet in LDS in wave order and its first wave adds
// into the gradient. Entries run longest (most groups) first so the many-split slabs' long
// blocks are not the launch's tail. Fixed summation order throughout: bit-reproducible, no atomics.
template <int G>
__global__ void __launch_bounds__(256) multi_splitk_reduce_kernel(MultiRed t) {
  // this workgroup's entry: the last one whose unit0 <= blockIdx.x (binary search: ~6 dependent
  // kernel-argument loads instead of up to 48 on a linear scan, before the first slab load)
  int k = 0;
  for (int lo = 0, hi = t.count - 1; lo <= hi;) {
    const int mid = (lo + hi) >> 1;
    if (t.e[mid].unit0 <= (int)blockIdx.x) {
      k = mid;
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  const float* slab = t.e[k].slab;
  float* out = t.e[k].out;
  const long n = t.e[k].n;
  const int splits = t.e[k].splits, groups = t.e[k].groups, vec = t.e[k].vec, wpc = t.e[k].wpc;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int chunk = (blockIdx.x - t.e[k].unit0) * (4 / wpc) + w / wpc, wj = w % wpc;
  __shared__ float4 red[4][64];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g = 0; g < groups; ++g) {
    const int s0 = g * G * wpc + wj * G;
    if (vec) {  // n % 4 == 0: lane owns 4 consecutive floats
      const long i4 = (long)chunk * 64 + lane;
      const bool ok = i4 * 4 < n;
      float4 v[G];
#pragma unroll
      for (int u = 0; u < G; ++u)
        v[u] = (ok && s0 + u < splits) ? reinterpret_cast<const float4*>(slab + (long)(s0 + u) * n)[i4]
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < G; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    } else {  // one float per lane
      const long i = (long)chunk * 64 + lane;
      const bool ok = i < n;
      float v[G];
#pragma unroll
      for (int u = 0; u < G; ++u) v[u] = (ok && s0 + u < splits) ? slab[(long)(s0 + u) * n + i] : 0.f;
#pragma unroll
      for (int u = 0; u < G; ++u) acc.x += v[u];
    }
  }
  if (wpc > 1) {
    red[w][lane] = acc;
    __syncthreads();
    if (wj > 0) return;
    for (int j = 1; j < wpc; ++j) {
      const float4 r = red[w + j][lane];
      acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
    }
  }
  if (vec) {
    const long i4 = (long)chunk * 64 + lane;
    if (i4 * 4 >= n) return;
    float4 c = reinterpret_cast<float4*>(out)[i4];
    c.x += acc.x; c.y += acc.y; c.z += acc.z; c.w += acc.w;
    reinterpret_cast<float4*>(out)[i4] = c;
  } else {
    const long i = (long)chunk * 64 + lane;
    if (i >= n) return;
    out[i] += acc.x;
  }
}

// slab loads in flight per wave and group (the summation order is fixed)
static constexpr int g_red_g = 16;

void multi_splitk_reduce(MultiRed t, hipStream_t s) {
  if (t.count <= 0) return;
  if (t.count > kMaxRed) throw std::runtime_error("multi_splitk_reduce: too many entries");
  for (int k = 0; k < t.count; ++k) {
    RedEnt& e = t.e[k];
    e.vec = (e.n % 4 == 0 && ((uintptr_t)e.slab % 16) == 0 && ((uintptr_t)e.out % 16) == 0) ? 1 : 0;
    // (a wave covers G splits per group: a second wave only pays once the splits exceed G)
    e.wpc = e.splits <= g_red_g ? 1 : (e.splits <= 2 * g_red_g ? 2 : 4);
    e.groups = (e.splits + g_red_g * e.wpc - 1) / (g_red_g * e.wpc);
  }
  // longest blocks first (stable: equal-length entries keep their queue order)
  std::stable_sort(t.e, t.e + t.count, [](const RedEnt& a, const RedEnt& b) { return a.groups > b.groups; });
  int units = 0;
  for (int k = 0; k < t.count; ++k) {
    RedEnt& e = t.e[k];
    const long per = e.vec ? 256 : 64;
    e.chunks = (int)((e.n + per - 1) / per);
    e.unit0 = units;
    const int cpb = 4 / e.wpc;
    units += (e.chunks + cpb - 1) / cpb;
  }
  if (g_red_g == 16)
    hipLaunchKernelGGL(multi_splitk_reduce_kernel<16>, dim3(units), dim3(256), 0, s, t);
  else
    hipLaunchKernelGGL(multi_splitk_reduce_kernel<8>, dim3(units), dim3(256), 0, s, t);
  DCNN_LAUNCH_CHECK();
}

// ----------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------
template <int BM, int BN, int BK, bool VEC>
static void launch_nt(const NtArgs& a, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, BK, VEC>), dim3(tiles), dim3(256), 0, s, a);
  DCNN_LAUNCH_CHECK();
}

int nt_tile_m(int M, int N) {
  // 128-row tiles unless that leaves the chip (256 CUs) under-filled
  const long t128 = (long)((M + 127) / 128) * ((N + 63) / 64);
  return t128 >= 512 ? 128 : 64;
}

void gemm_nt(const NtArgs& a, hipStream_t s) {
  const bool conv = a.mode != kPlain;
  const bool vec = conv ? (a.cs % 32 == 0 && a.K % 32 == 0) : (a.K % 8 == 0 && a.lda % 8 == 0);
  const bool vecb = a.ldb % 8 == 0 && a.K % 8 == 0;
  const bool v = vec && vecb;
  const int bk = (!v || (conv && a.cs % 64 != 0) || (!conv && a.K % 64 != 0)) ? 32 : 64;
  const int bm = nt_tile_m(a.M, a.N);
  const long tiles_big = (long)((a.M + bm - 1) / bm) * ((a.N + 127) / 128);
  const int bn = (a.N >= 128 && tiles_big >= 256) ? 128 : 64;
#define DCNN_NT(BM, BN, BK, V) if (bm == BM && bn == BN && bk == BK && v == V) return launch_nt<BM, BN, BK, V>(a, s)
  DCNN_NT(128, 128, 64, true);
  DCNN_NT(128, 64, 64, true);
  DCNN_NT(64, 128, 64, true);
  DCNN_NT(64, 64, 64, true);
  DCNN_NT(128, 128, 32, true);
  DCNN_NT(128, 64, 32, true);
  DCNN_NT(64, 128, 32, true);
  DCNN_NT(64, 64, 32, true);
  DCNN_NT(128, 64, 32, false);
  DCNN_NT(64, 64, 32, false);
  DCNN_NT(128, 128, 32, false);
  DCNN_NT(64, 128, 32, false);
#undef DCNN_NT
  throw std::runtime_error("gemm_nt: no kernel variant for configuration");
}

// rows of the partial-statistics slab produced by gemm_nt for a given problem
int gemm_nt_stat_rows(int M, int N) { return (M + nt_tile_m(M, N) - 1) / nt_tile_m(M, N); }

template <int BM, int BN, int BK, bool VEC>
static void launch_tn(TnArgs a, int splits, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_tn_kernel<BM, BN, BK, VEC>), dim3(tiles * splits), dim3(256), 0, s, a);
  DCNN_LAUNCH_CHECK();
}

// Choose the split count for the weight-gradient GEMM: enough workgroups to fill 256 CUs
// (~2 per CU) while keeping >= 4 K-steps per split and the fp32 slab bounded.
int gemm_tn_splits(int M, int N, int P) {
  const int bm = M >= 128 ? 128 : 64, bn = N >= 128 ? 128 : 64;
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  long splits = (512 + tiles - 1) / tiles;
  // at least 4 K-steps (256 reduction rows) per split; a grid of few tiles (a classifier's weight
  // gradient: 200 x 512 over the batch, 8 tiles) may go down to one K-step per split instead of
  // running 8 workgroups through the whole batch (ResNet-18 fc: 17.7 us at one split)
  const long min_k = tiles < 32 ? 64 : 64 * 4;
  const long max_by_k = P / min_k > 0 ? P / min_k : 1;
  if (splits > max_by_k) splits = max_by_k;
  const long max_by_mem = (64l << 20) / (4l * M * N) > 0 ? (64l << 20) / (4l * M * N) : 1;
  if (splits > max_by_mem) splits = max_by_mem;
  if (splits < 1) splits = 1;
  if (splits > 128) splits = 128;
  return (int)splits;
}

void gemm_tn(TnArgs a, int splits, hipStream_t s) {
  const bool conv = a.mode == kConvFwd;
  const int bm = a.M >= 128 ? 128 : 64;
  int bn = a.N >= 128 ? 128 : 64;
  if (conv) while (bn > 32 && a.cs % bn != 0) bn >>= 1;
  const bool v = a.M % 8 == 0 && (conv ? a.cs % bn == 0 : (a.N % 8 == 0 && a.ldx % 8 == 0));
  if (!v) bn = a.N >= 128 ? 128 : 64;
  const int per = (a.P + splits - 1) / splits;
  a.k_per_split = ((per + 63) / 64) * 64;
#define DCNN_TN(BM, BN, V) if (bm == BM && bn == BN && v == V) return launch_tn<BM, BN, 64, V>(a, splits, s)
  DCNN_TN(128, 128, true);
  DCNN_TN(128, 64, true);
  DCNN_TN(128, 32, true);
  DCNN_TN(64, 128, true);
  DCNN_TN(64, 64, true);
  DCNN_TN(64, 32, true);
  DCNN_TN(128, 128, false);
  DCNN_TN(128, 64, false);
  DCNN_TN(64, 128, false);
  DCNN_TN(64, 64, false);
#undef DCNN_TN
  throw std::runtime_error("gemm_tn: no kernel variant");
}

void splitk_reduce2(const float* slab, float* out, long n, const float* bslab, float* bout, long nb, int splits,
                    int accumulate, hipStream_t s) {
  const long n4 = n / 4 + 1;
  const int gxa = grid_for(n4, 256, 4096);
  const int gxb = nb > 0 ? grid_for(nb / 4 + 1, 256, 64) : 0;
  const SplitkSeg a{slab, out, n}, b{bslab, bout, nb > 0 ? nb : 0};
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gxa + gxb), dim3(256), 0, s, a, b, gxa, splits, accumulate);
  DCNN_LAUNCH_CHECK();
}

void splitk_reduce(const float* slab, float* out, long n, int splits, int accumulate, hipStream_t s) {
  splitk_reduce2(slab, out, n, nullptr, nullptr, 0, splits, accumulate, s);
}

}  // namespace dcnn
