// fp32 implicit-GEMM convolution / dense kernels on CDNA4 MFMA.
//
// The fp32 compute path (the reference's only precision; BASELINE config "CIFAR-10 ResNet-9
// fp32") uses the same gathered-GEMM formulation and host-side tap tables as the bf16 v2
// kernels (gemm2.hip) — conv forward, phase-decomposed dgrad and dense share one NT kernel
// family, weight gradients one split-K TN kernel family — with fp32 operands end to end:
//
// * Forward / dgrad: 128 x 128 or 128 x 64 tiles on v_mfma_f32_32x32x2_f32 where the grid still
//   fills the chip with them, else 64 x 64 tiles on v_mfma_f32_16x16x4_f32 (2x2 waves, 32x32 per
//   wave); BK = 16 reduction elements per stage, global float4 loads register-staged one stage
//   ahead (loads of tile k+1 overlap the MFMAs of tile k), the tap of a 16-multiple channel block
//   looked up wave-uniformly.
// * Weight gradient: pixel-major LDS tiles (see gemm_t2f_wide_kernel), 64 / 128 per side.
// * Padding / out-of-image taps are zero-filled from a per-row tap-validity mask.
// * Epilogue: bias, residual add, ReLU and per-channel BatchNorm (sum, sum^2) partials, with
//   the strided output-row scatter of a dgrad phase.
#include <cstdlib>

#include "common.h"
#include "api.h"

namespace dcnn {

namespace {
constexpr int FBM = 64, FBN = 64, FBK = 16, FPITCH = FBK + 4;  // LDS row pitch (floats): conflict-free b128 reads

__device__ __forceinline__ int xcd_remap_f(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ f32x4 mfma4(const float4& a, const float4& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}
}  // namespace

// C[m][n] = sum_{t, c} Src[pix(m) + tap t][c] * B[n][tap_b[t] + c]   (G2Args semantics, fp32)
__global__ void __launch_bounds__(256, 2) gemm_g2f_kernel(G2Args p) {
  prefetch_kernargs<sizeof(G2Args)>();
  __shared__ __attribute__((aligned(16))) float As[2][FBM * FPITCH];
  __shared__ __attribute__((aligned(16))) float Bs[2][FBN * FPITCH];
  __shared__ float red[2][4][FBN];  // per M-wave: shifted (sum, sum^2), pivot, count
  const float* A = reinterpret_cast<const float*>(p.A);
  const float* B = reinterpret_cast<const float*>(p.B);
  float* C = reinterpret_cast<float*>(p.C);
  const float* R = reinterpret_cast<const float*>(p.residual);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (p.N + FBN - 1) / FBN;
  const int lt = xcd_remap_f(blockIdx.x, gridDim.x);
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int m0 = tm * FBM, n0 = tn * FBN;
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;

  // this thread loads row lr, float4 chunk lc (4 chunks of 4 floats = BK 16)
  const int lr = tid >> 2, lc = tid & 3;
  long a_base = 0;
  uint64_t a_mask = 0;
  {
    const int m = m0 + lr;
    if (m < p.M) {
      const int ghw = p.GH * p.GW;
      const int img = m / ghw, rem = m - img * ghw;
      const int gy = rem / p.GW, gx = rem - gy * p.GW;
      const int y0 = gy * p.SY, x0 = gx * p.SX;
      a_base = (((long)img * p.H + y0) * p.W + x0) * p.Cs;
      for (int t = 0; t < p.ntaps; ++t) {
        const int sy = y0 + p.tap_dy[t], sx = x0 + p.tap_dx[t];
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W) a_mask |= (1ull << t);
      }
    }
  }
  const int bn_row = n0 + lr;
  const bool b_ok = bn_row < p.N;
  const long b_base = (long)bn_row * p.ldb;
  const bool vec = (p.Cs & 3) == 0, uni = p.Cs % FBK == 0;

  auto load = [&](int k0, float4& ra, float4& rb) {
    float va[4], vb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) { va[e] = 0.f; vb[e] = 0.f; }
    const int k = k0 + lc * 4;
    if (vec) {  // the 4 elements share one tap
      // (a 16-multiple channel count: the whole K block shares one tap -> wave-uniform t, a
      // scalar division and scalar loads of the tap tables)
      const int tu = k0 / p.Cs;
      const int t = uni ? tu : k / p.Cs, c = uni ? k0 - tu * p.Cs + lc * 4 : k - t * p.Cs;
      if (t < p.ntaps) {
        if ((a_mask >> t) & 1ull) {
          const float4 v = *reinterpret_cast<const float4*>(A + a_base + p.tap_srcoff[t] + c);
          va[0] = v.x; va[1] = v.y; va[2] = v.z; va[3] = v.w;
        }
        if (b_ok) {
          const float4 v = *reinterpret_cast<const float4*>(B + b_base + p.tap_b[t] + c);
          vb[0] = v.x; vb[1] = v.y; vb[2] = v.z; vb[3] = v.w;
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = k + e, t = kk / p.Cs, c = kk - t * p.Cs;
        if (t < p.ntaps) {
          if ((a_mask >> t) & 1ull) va[e] = A[a_base + p.tap_srcoff[t] + c];
          if (b_ok) vb[e] = B[b_base + p.tap_b[t] + c];
        }
      }
    }
    ra = make_float4(va[0], va[1], va[2], va[3]);
    rb = make_float4(vb[0], vb[1], vb[2], vb[3]);
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int K = p.ntaps * p.Cs;
  const int nk = (K + FBK - 1) / FBK;
  float4 ra, rb;
  load(0, ra, rb);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    *reinterpret_cast<float4*>(&As[cur][lr * FPITCH + lc * 4]) = ra;
    *reinterpret_cast<float4*>(&Bs[cur][lr * FPITCH + lc * 4]) = rb;
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * FBK, ra, rb);
    const int g = lane >> 4;
    float4 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      a[i] = *reinterpret_cast<const float4*>(&As[cur][(wm * 32 + i * 16 + (lane & 15)) * FPITCH + g * 4]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[j] = *reinterpret_cast<const float4*>(&Bs[cur][(wn * 32 + j * 16 + (lane & 15)) * FPITCH + g * 4]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(a[i], b[j], acc[i][j]);
    cur ^= 1;
  }

  // ---- epilogue straight from the accumulators: lane owns column (lane&15) of each subtile ----
  // Forward BatchNorm statistics: per (M-wave, column) the values are summed about a pivot (the
  // wave's first row of the column), reduced over the lane groups by a fixed butterfly, and the
  // two M-waves are merged with Chan's update into a (count, mean, M2) triple. No atomics.
  const int ghw = p.GH * p.GW;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 32 + j * 16 + (lane & 15);
    const bool cok = col < p.N;
    const float bv = (p.bias && cok) ? p.bias[col] : 0.f;
    const float piv = __shfl(acc[0][j][0] + bv, lane & 15, 64);
    float s = 0.f, q = 0.f, n = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.M || !cok) continue;
        const int img = m / ghw, rem = m - img * ghw;
        const int gy = rem / p.GW, gx = rem - gy * p.GW;
        const long orow = ((long)img * p.OH + gy * p.OSY + p.ORY) * p.OW + gx * p.OSX + p.ORX;
        float v = acc[i][j][r] + bv;
        if (R) v += R[orow * p.ldc + col];
        if (p.relu) v = fmaxf(v, 0.f);
        C[orow * p.ldc + col] = v;
        const float d = v - piv;
        s += d;
        q += d * d;
        n += 1.f;
      }
    if (p.stats) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      n += __shfl_xor(n, 16, 64);
      n += __shfl_xor(n, 32, 64);
      if (lane < 16) {
        const int c = wn * 32 + j * 16 + lane;
        red[wm][0][c] = s;
        red[wm][1][c] = q;
        red[wm][2][c] = piv;
        red[wm][3][c] = n;
      }
    }
  }
  if (p.stats) {
    __syncthreads();
    if (tid < FBN && n0 + tid < p.N) {
      Welford t = welford_from_shifted(red[0][3][tid], red[0][2][tid], red[0][0][tid], red[0][1][tid]);
      t = welford_merge(t, welford_from_shifted(red[1][3][tid], red[1][2][tid], red[1][0][tid], red[1][1][tid]));
      store_welford(p.stats, tm, p.N, n0 + tid, t);
    }
  }
}

// Wide-tile variant of gemm_g2f_kernel for the grids that fill the chip with it: a BM x BN = 128 x
// 128 output tile, 4 waves of 64 x 64, each wave 2 x 2 tiles of v_mfma_f32_32x32x2_f32 (16
// accumulators each). Twice the output columns share every gathered A row and twice the rows
// every B row, so the tap-gather loads per FLOP halve (the 64 x 64 kernel is load-bound on the
// ResNet shapes). K order: k-block rows are read as two float4 per lane (lane half h holds
// k = 8h .. 8h + 7 of the block); MFMA step s takes k = s from half 0 and k = 8 + s from half 1 for
// BOTH operands, so every k is summed once (the order differs from the 16x16x4 kernel: exact f32
// arithmetic, a different fma chain).
// (BK = 32 measured slower: ResNet-9 fp32 15.3k -> 15.1k, ResNet-18 17.0k -> 16.5k img/s)
template <int BM, int BN, int BK = FBK>
__global__ void __launch_bounds__(256, 2) gemm_g2f_wide_kernel(G2Args p) {
  constexpr int WM = BM / 2, WN = BN / 2;     // per-wave tile
  constexpr int TM = WM / 32, TN = WN / 32;   // 32x32 MFMA tiles per wave
  constexpr int PITCH = BK + 4;               // LDS row pitch (floats)
  constexpr int CH = BK / 4, RP = 256 / CH;   // float4 chunks per row, rows per loader pass
  constexpr int AR = BM / RP, BR = BN / RP;   // loader rows per thread
  __shared__ __attribute__((aligned(16))) float As[2][BM * PITCH];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * PITCH];
  __shared__ float red[2][4][BN];
  const float* A = reinterpret_cast<const float*>(p.A);
  const float* B = reinterpret_cast<const float*>(p.B);
  float* C = reinterpret_cast<float*>(p.C);
  const float* R = reinterpret_cast<const float*>(p.residual);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int lt = xcd_remap_f(blockIdx.x, gridDim.x);
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;

  const int lr = tid / CH, lc = tid % CH;  // loader: rows lr + RP r, float4 chunk lc
  long a_base[AR];
  uint64_t a_mask[AR];
#pragma unroll
  for (int r = 0; r < AR; ++r) {
    a_base[r] = 0;
    a_mask[r] = 0;
    const int m = m0 + lr + RP * r;
    if (m < p.M) {
      const int ghw = p.GH * p.GW;
      const int img = m / ghw, rem = m - img * ghw;
      const int gy = rem / p.GW, gx = rem - gy * p.GW;
      const int y0 = gy * p.SY, x0 = gx * p.SX;
      a_base[r] = (((long)img * p.H + y0) * p.W + x0) * p.Cs;
      for (int t = 0; t < p.ntaps; ++t) {
        const int sy = y0 + p.tap_dy[t], sx = x0 + p.tap_dx[t];
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W) a_mask[r] |= (1ull << t);
      }
    }
  }
  bool b_ok[BR];
  long b_base[BR];
#pragma unroll
  for (int r = 0; r < BR; ++r) {
    const int n = n0 + lr + RP * r;
    b_ok[r] = n < p.N;
    b_base[r] = (long)n * p.ldb;
  }
  const bool vec = (p.Cs & 3) == 0, uni = p.Cs % BK == 0;

  auto load = [&](int k0, float4 (&ra)[AR], float4 (&rb)[BR]) {
    const int k = k0 + lc * 4;
#pragma unroll
    for (int r = 0; r < AR; ++r) ra[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < BR; ++r) rb[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec) {  // the 4 elements share one tap (BK-multiple channels: wave-uniform, as above)
      const int tu = k0 / p.Cs;
      const int t = uni ? tu : k / p.Cs, c = uni ? k0 - tu * p.Cs + lc * 4 : k - t * p.Cs;
      if (t < p.ntaps) {
#pragma unroll
        for (int r = 0; r < AR; ++r)
          if ((a_mask[r] >> t) & 1ull) ra[r] = *reinterpret_cast<const float4*>(A + a_base[r] + p.tap_srcoff[t] + c);
#pragma unroll
        for (int r = 0; r < BR; ++r)
          if (b_ok[r]) rb[r] = *reinterpret_cast<const float4*>(B + b_base[r] + p.tap_b[t] + c);
      }
    } else {
      float va[AR][4], vb[BR][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = k + e, t = kk / p.Cs, c = kk - t * p.Cs;
#pragma unroll
        for (int r = 0; r < AR; ++r) va[r][e] = (t < p.ntaps && ((a_mask[r] >> t) & 1ull)) ? A[a_base[r] + p.tap_srcoff[t] + c] : 0.f;
#pragma unroll
        for (int r = 0; r < BR; ++r) vb[r][e] = (t < p.ntaps && b_ok[r]) ? B[b_base[r] + p.tap_b[t] + c] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < AR; ++r) ra[r] = make_float4(va[r][0], va[r][1], va[r][2], va[r][3]);
#pragma unroll
      for (int r = 0; r < BR; ++r) rb[r] = make_float4(vb[r][0], vb[r][1], vb[r][2], vb[r][3]);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int K = p.ntaps * p.Cs;
  const int nk = (K + BK - 1) / BK;
  float4 ra[AR], rb[BR];
  load(0, ra, rb);
  int cur = 0;
  const int h = lane >> 5, l32 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
    for (int r = 0; r < AR; ++r) *reinterpret_cast<float4*>(&As[cur][(lr + RP * r) * PITCH + lc * 4]) = ra[r];
#pragma unroll
    for (int r = 0; r < BR; ++r) *reinterpret_cast<float4*>(&Bs[cur][(lr + RP * r) * PITCH + lc * 4]) = rb[r];
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * BK, ra, rb);
#pragma unroll
    for (int kb = 0; kb < BK / 16; ++kb) {  // 16-wide k blocks, each in the two-half order above
      float a[TM][8], b[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = &As[cur][(wm * WM + i * 32 + l32) * PITCH + kb * 16 + h * 8];
        const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
        a[i][0] = x0.x; a[i][1] = x0.y; a[i][2] = x0.z; a[i][3] = x0.w;
        a[i][4] = x1.x; a[i][5] = x1.y; a[i][6] = x1.z; a[i][7] = x1.w;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* src = &Bs[cur][(wn * WN + j * 32 + l32) * PITCH + kb * 16 + h * 8];
        const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
        b[j][0] = x0.x; b[j][1] = x0.y; b[j][2] = x0.z; b[j][3] = x0.w;
        b[j][4] = x1.x; b[j][5] = x1.y; b[j][6] = x1.z; b[j][7] = x1.w;
      }
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s2], b[j][s2], acc[i][j], 0, 0, 0);
    }
    cur ^= 1;
  }

  // ---- epilogue from the accumulators: lane owns column l32 of each 32x32 tile, rows
  // (e & 3) + 8 (e >> 2) + 4 h of register e
  const int ghw = p.GH * p.GW;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn * WN + j * 32 + l32;
    const int col = n0 + cl;
    const bool cok = col < p.N;
    const float bv = (p.bias && cok) ? p.bias[col] : 0.f;
    // pivot: the wave's first row of the column (register 0 of lane half 0)
    const float piv = __shfl(acc[0][j][0] + bv, l32, 64);
    float s = 0.f, q = 0.f, n = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m >= p.M || !cok) continue;
        const int img = m / ghw, rem = m - img * ghw;
        const int gy = rem / p.GW, gx = rem - gy * p.GW;
        const long orow = ((long)img * p.OH + gy * p.OSY + p.ORY) * p.OW + gx * p.OSX + p.ORX;
        float v = acc[i][j][e] + bv;
        if (R) v += R[orow * p.ldc + col];
        if (p.relu) v = fmaxf(v, 0.f);
        C[orow * p.ldc + col] = v;
        const float d = v - piv;
        s += d;
        q += d * d;
        n += 1.f;
      }
    if (p.stats) {
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 32, 64);
      n += __shfl_xor(n, 32, 64);
      if (h == 0) {
        red[wm][0][cl] = s;
        red[wm][1][cl] = q;
        red[wm][2][cl] = piv;
        red[wm][3][cl] = n;
      }
    }
  }
  if (p.stats) {
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c >= p.N) continue;
      Welford t = welford_from_shifted(red[0][3][c], red[0][2][c], red[0][0][c], red[0][1][c]);
      t = welford_merge(t, welford_from_shifted(red[1][3][c], red[1][2][c], red[1][0][c], red[1][1][c]));
      store_welford(p.stats, tm, p.N, n0 + c, t);
    }
  }
}

// Exact-fp32 weight gradient, dW[m][n] (+ bias grad) = sum_p dY[p][m] * X[gather(p, tap(n))][c(n)]
// over this split's pixels: a BM x BN (64 / 128) dW tile per split on v_mfma_f32_32x32x2_f32
// (4 waves of BM/2 x BN/2). Both operands arrive pixel-major (a pixel's dY row, a pixel's gathered X
// row), so the LDS tiles are kept pixel-major too — [k][m] / [k][n], float4 stores along m / n
// (conflict-free) — and every MFMA operand is one ds_read_b32: lane half h reads pixel 2s + h of
// the 16-pixel tile, lane l32 its column. The next tile's global loads are issued right after the
// barrier and land in registers while this tile's 32 MFMAs run (double-buffered LDS, one barrier
// per tile); each thread's tap / channel / validity terms are fixed per column and its pixel
// coordinates advance incrementally (no divisions in the loop).
template <int BM, int BN>
__global__ void __launch_bounds__(256, 2) gemm_t2f_wide_kernel(T2Args p) {
  prefetch_kernargs<sizeof(T2Args)>();
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int AQ = BM / 64, BQ = BN / 64;  // float4 column groups per thread (16 threads x 4 cols per pass)
  constexpr int PA = BM + 4, PB = BN + 4;    // LDS row pitch (floats)
  __shared__ __attribute__((aligned(16))) float As[2][FBK * PA];  // [k][m]
  __shared__ __attribute__((aligned(16))) float Bs[2][FBK * PB];  // [k][n]
  const float* dY = reinterpret_cast<const float*>(p.dY);
  const float* X = reinterpret_cast<const float*>(p.X);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int lt = xcd_remap_f(blockIdx.x, gridDim.x);
  const int split = lt / tiles, tt = lt % tiles;
  const int tm = tt / tiles_n, tn = tt % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const long pbeg = (long)split * p.k_per_split;
  const long pend = pbeg + p.k_per_split < p.P ? pbeg + p.k_per_split : p.P;
  const int lk = tid >> 4, lq = tid & 15;  // loader: pixel lk of the tile, columns 4 lq + 64 r
  // per-column terms, fixed over the loop
  bool a_vec[AQ];
  int a_col[AQ];
#pragma unroll
  for (int r = 0; r < AQ; ++r) {
    a_col[r] = m0 + lq * 4 + 64 * r;
    a_vec[r] = (p.ldy & 3) == 0 && a_col[r] + 3 < p.M;
  }
  const bool b_vec = (p.Cs & 3) == 0;
  int b_dy[BQ][4], b_dx[BQ][4], b_c[BQ][4];
  bool b_ok[BQ][4];
#pragma unroll
  for (int r = 0; r < BQ; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + lq * 4 + 64 * r + e;
      b_ok[r][e] = n < p.N;
      const int t = b_ok[r][e] ? n / p.Cs : 0;
      b_c[r][e] = n - t * p.Cs;
      b_dy[r][e] = p.tap_dy[t];
      b_dx[r][e] = p.tap_dx[t];
    }
  // this thread's pixel: pbeg + lk, then + FBK per tile
  const int ghw = p.GH * p.GW;
  long pix = pbeg + lk;
  int img = (int)(pix / ghw), gy, gx;
  {
    const int rem = (int)(pix - (long)img * ghw);
    gy = rem / p.GW;
    gx = rem - gy * p.GW;
  }
  auto advance = [&]() {
    pix += FBK;
    gx += FBK;
    while (gx >= p.GW) {
      gx -= p.GW;
      if (++gy == p.GH) {
        gy = 0;
        ++img;
      }
    }
  };
  auto load = [&](float4 (&ra)[AQ], float4 (&rb)[BQ]) {
#pragma unroll
    for (int r = 0; r < AQ; ++r) ra[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < BQ; ++r) rb[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (pix >= pend) return;
#pragma unroll
    for (int r = 0; r < AQ; ++r) {
      const float* src = dY + pix * p.ldy + a_col[r];
      if (a_vec[r]) {
        ra[r] = *reinterpret_cast<const float4*>(src);
      } else {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = a_col[r] + e < p.M ? src[e] : 0.f;
        ra[r] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    const int y0 = gy * p.SY, x0 = gx * p.SX;
    const long ibase = (long)img * p.H;
#pragma unroll
    for (int r = 0; r < BQ; ++r) {
      if (b_vec && b_ok[r][3]) {  // the 4 columns share one tap
        const int sy = y0 + b_dy[r][0], sx = x0 + b_dx[r][0];
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W)
          rb[r] = *reinterpret_cast<const float4*>(X + ((ibase + sy) * p.W + sx) * p.Cs + b_c[r][0]);
      } else {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int sy = y0 + b_dy[r][e], sx = x0 + b_dx[r][e];
          v[e] = (b_ok[r][e] && sy >= 0 && sy < p.H && sx >= 0 && sx < p.W)
                     ? X[((ibase + sy) * p.W + sx) * p.Cs + b_c[r][e]]
                     : 0.f;
        }
        rb[r] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };

  float bias_acc = 0.f;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int h = lane >> 5, l32 = lane & 31;
  const int nt = (int)((pend - pbeg + FBK - 1) / FBK);
  float4 ra[AQ], rb[BQ];
  load(ra, rb);
  int cur = 0;
  for (int it = 0; it < nt; ++it) {
#pragma unroll
    for (int r = 0; r < AQ; ++r) *reinterpret_cast<float4*>(&As[cur][lk * PA + lq * 4 + 64 * r]) = ra[r];
#pragma unroll
    for (int r = 0; r < BQ; ++r) *reinterpret_cast<float4*>(&Bs[cur][lk * PB + lq * 4 + 64 * r]) = rb[r];
    __syncthreads();
    if (it + 1 < nt) {
      advance();
      load(ra, rb);
    }
    if (p.bias_slab && tn == 0 && tid < BM) {
#pragma unroll
      for (int k = 0; k < FBK; ++k) bias_acc += As[cur][k * PA + tid];
    }
    const float* Ac = &As[cur][h * PA + wm * WM + l32];
    const float* Bc = &Bs[cur][h * PB + wn * WN + l32];
#pragma unroll
    for (int s2 = 0; s2 < FBK / 2; ++s2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = Ac[2 * s2 * PA + i * 32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bc[2 * s2 * PB + j * 32];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    cur ^= 1;
  }
  float* out = p.slab + (long)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 32 + l32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row < p.M && col < p.N) out[(long)row * p.N + col] = acc[i][j][e];
      }
    }
  if (p.bias_slab && tn == 0 && tid < BM && m0 + tid < p.M) p.bias_slab[(long)split * p.M + m0 + tid] = bias_acc;
}

// ------------------------------------------------------------------------------------------
// fp32 GEMMs on bf16 MFMA with split precision ("3xbf16"): every fp32 operand x is split once,
// when its tile is staged into LDS, into hi = bf16(x) and lo = bf16(x - hi), and each 16x16x32
// product block is accumulated in fp32 as  a_hi*b_hi + a_hi*b_lo + a_lo*b_hi  (the a_lo*b_lo
// term, ~2^-16 relative, is dropped). That is 16 significant bits per operand instead of 24, at
// 3 bf16 MFMAs = 3/16 of the cycles of the exact 16x16x4 f32 MFMA chain for the same K: the fp32
// path's GEMMs become ~4-5x cheaper in matrix-pipe time. Same tiling, tap gathers, epilogue
// (bias / residual / ReLU / BN statistics) and split-K slabs as the exact kernels above.
// Opt-in (set_f32_mode(1), `bench.py --f32-mode split`): on ResNet-18/ResNet-9 fp32 these gathered-GEMM
// kernels are bound by their tap-gather loads, not the matrix pipe, so the split forward/dgrad
// kernel was 18% faster and the split wgrad 26% slower than exact (profiles/fp32_split_r2.md) —
// the exact f32 MFMA path stays the default. tests/test_gpu_kernels.py bounds the split error
// against an fp64 reference (4.5e-6 relative on a K = 4608 conv).
// ------------------------------------------------------------------------------------------
namespace {
constexpr int XBK = 32, XP = XBK + 8;  // bf16 row pitch 80 B: conflict-free ds_read_b128 over 16 rows
int g_f32_mode = -1;                   // 0 exact f32 MFMA (default), 1 split bf16 (3 MFMAs)

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16 h = (bf16)v[e];
    hi[e] = h;
    lo[e] = (bf16)(v[e] - (float)h);
  }
}

__device__ __forceinline__ f32x4 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
  return c;
}
}  // namespace

__global__ void __launch_bounds__(256, 2) gemm_g2x_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) bf16 Ah[2][FBM * XP], Al[2][FBM * XP];
  __shared__ __attribute__((aligned(16))) bf16 Bh[2][FBN * XP], Bl[2][FBN * XP];
  __shared__ float red[2][4][FBN];
  const float* A = reinterpret_cast<const float*>(p.A);
  const float* B = reinterpret_cast<const float*>(p.B);
  float* C = reinterpret_cast<float*>(p.C);
  const float* R = reinterpret_cast<const float*>(p.residual);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (p.N + FBN - 1) / FBN;
  const int lt = xcd_remap_f(blockIdx.x, gridDim.x);
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int m0 = tm * FBM, n0 = tn * FBN;
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;

  // this thread stages row lr, k chunk lc of 8 (4 chunks = XBK 32)
  const int lr = tid >> 2, lc = tid & 3;
  long a_base = 0;
  uint64_t a_mask = 0;
  {
    const int m = m0 + lr;
    if (m < p.M) {
      const int ghw = p.GH * p.GW;
      const int img = m / ghw, rem = m - img * ghw;
      const int gy = rem / p.GW, gx = rem - gy * p.GW;
      const int y0 = gy * p.SY, x0 = gx * p.SX;
      a_base = (((long)img * p.H + y0) * p.W + x0) * p.Cs;
      for (int t = 0; t < p.ntaps; ++t) {
        const int sy = y0 + p.tap_dy[t], sx = x0 + p.tap_dx[t];
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W) a_mask |= (1ull << t);
      }
    }
  }
  const int bn_row = n0 + lr;
  const bool b_ok = bn_row < p.N;
  const long b_base = (long)bn_row * p.ldb;
  const bool vec = (p.Cs & 3) == 0;

  auto load = [&](int k0, float (&va)[8], float (&vb)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { va[e] = 0.f; vb[e] = 0.f; }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k0 + lc * 8 + h * 4;
      if (vec) {  // 4 elements share one tap
        const int t = k / p.Cs, c = k - t * p.Cs;
        if (t < p.ntaps) {
          if ((a_mask >> t) & 1ull) {
            const float4 v = *reinterpret_cast<const float4*>(A + a_base + p.tap_srcoff[t] + c);
            va[h * 4 + 0] = v.x; va[h * 4 + 1] = v.y; va[h * 4 + 2] = v.z; va[h * 4 + 3] = v.w;
          }
          if (b_ok) {
            const float4 v = *reinterpret_cast<const float4*>(B + b_base + p.tap_b[t] + c);
            vb[h * 4 + 0] = v.x; vb[h * 4 + 1] = v.y; vb[h * 4 + 2] = v.z; vb[h * 4 + 3] = v.w;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = k + e, t = kk / p.Cs, c = kk - t * p.Cs;
          if (t < p.ntaps) {
            if ((a_mask >> t) & 1ull) va[h * 4 + e] = A[a_base + p.tap_srcoff[t] + c];
            if (b_ok) vb[h * 4 + e] = B[b_base + p.tap_b[t] + c];
          }
        }
      }
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int K = p.ntaps * p.Cs;
  const int nk = (K + XBK - 1) / XBK;
  float va[8], vb[8];
  load(0, va, vb);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    {
      bf16x8 h, l;
      split8(va, h, l);
      *reinterpret_cast<bf16x8*>(&Ah[cur][lr * XP + lc * 8]) = h;
      *reinterpret_cast<bf16x8*>(&Al[cur][lr * XP + lc * 8]) = l;
      split8(vb, h, l);
      *reinterpret_cast<bf16x8*>(&Bh[cur][lr * XP + lc * 8]) = h;
      *reinterpret_cast<bf16x8*>(&Bl[cur][lr * XP + lc * 8]) = l;
    }
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * XBK, va, vb);
    const int g = lane >> 4;
    bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = (wm * 32 + i * 16 + (lane & 15)) * XP + g * 8;
      ah[i] = *reinterpret_cast<const bf16x8*>(&Ah[cur][o]);
      al[i] = *reinterpret_cast<const bf16x8*>(&Al[cur][o]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o = (wn * 32 + j * 16 + (lane & 15)) * XP + g * 8;
      bh[j] = *reinterpret_cast<const bf16x8*>(&Bh[cur][o]);
      bl[j] = *reinterpret_cast<const bf16x8*>(&Bl[cur][o]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma3(ah[i], al[i], bh[j], bl[j], acc[i][j]);
    cur ^= 1;
  }

  // ---- epilogue (identical to gemm_g2f_kernel) ----
  const int ghw = p.GH * p.GW;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 32 + j * 16 + (lane & 15);
    const bool cok = col < p.N;
    const float bv = (p.bias && cok) ? p.bias[col] : 0.f;
    const float piv = __shfl(acc[0][j][0] + bv, lane & 15, 64);
    float s = 0.f, q = 0.f, n = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.M || !cok) continue;
        const int img = m / ghw, rem = m - img * ghw;
        const int gy = rem / p.GW, gx = rem - gy * p.GW;
        const long orow = ((long)img * p.OH + gy * p.OSY + p.ORY) * p.OW + gx * p.OSX + p.ORX;
        float v = acc[i][j][r] + bv;
        if (R) v += R[orow * p.ldc + col];
        if (p.relu) v = fmaxf(v, 0.f);
        C[orow * p.ldc + col] = v;
        const float d = v - piv;
        s += d;
        q += d * d;
        n += 1.f;
      }
    if (p.stats) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      n += __shfl_xor(n, 16, 64);
      n += __shfl_xor(n, 32, 64);
      if (lane < 16) {
        const int c = wn * 32 + j * 16 + lane;
        red[wm][0][c] = s;
        red[wm][1][c] = q;
        red[wm][2][c] = piv;
        red[wm][3][c] = n;
      }
    }
  }
  if (p.stats) {
    __syncthreads();
    if (tid < FBN && n0 + tid < p.N) {
      Welford t = welford_from_shifted(red[0][3][tid], red[0][2][tid], red[0][0][tid], red[0][1][tid]);
      t = welford_merge(t, welford_from_shifted(red[1][3][tid], red[1][2][tid], red[1][0][tid], red[1][1][tid]));
      store_welford(p.stats, tm, p.N, n0 + tid, t);
    }
  }
}

// split-precision weight gradient: thread (column tcol = tid & 63, k group tk = tid >> 6 of 8
// pixels) loads 8 pixels of one dY column and of one gathered X column (coalesced across the
// wave's 64 lanes), splits them and stores contiguous bf16x8 k-runs.
__global__ void __launch_bounds__(256, 2) gemm_t2x_kernel(T2Args p) {
  __shared__ __attribute__((aligned(16))) bf16 Ah[FBM * XP], Al[FBM * XP];
  __shared__ __attribute__((aligned(16))) bf16 Bh[FBN * XP], Bl[FBN * XP];
  const float* dY = reinterpret_cast<const float*>(p.dY);
  const float* X = reinterpret_cast<const float*>(p.X);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_m = (p.M + FBM - 1) / FBM, tiles_n = (p.N + FBN - 1) / FBN;
  const int tiles = tiles_m * tiles_n;
  const int lt = xcd_remap_f(blockIdx.x, gridDim.x);
  const int split = lt / tiles, tt = lt % tiles;
  const int tm = tt / tiles_n, tn = tt % tiles_n;
  const int m0 = tm * FBM, n0 = tn * FBN;
  const long pbeg = (long)split * p.k_per_split;
  const long pend = pbeg + p.k_per_split < p.P ? pbeg + p.k_per_split : p.P;

  const int tcol = tid & 63, tk = tid >> 6;
  const int am = m0 + tcol, bn = n0 + tcol;
  const bool aok = am < p.M, bok = bn < p.N;
  const int bt = bok ? bn / p.Cs : 0, bc = bok ? bn - bt * p.Cs : 0;
  const int bdy = bok ? p.tap_dy[bt] : 0, bdx = bok ? p.tap_dx[bt] : 0;
  float bias_acc = 0.f;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ghw = p.GH * p.GW;
  for (long k0 = pbeg; k0 < pend; k0 += XBK) {
    float va[8], vb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long pix = k0 + tk * 8 + e;
      va[e] = 0.f;
      vb[e] = 0.f;
      if (pix < pend) {
        if (aok) va[e] = dY[pix * p.ldy + am];
        if (bok) {
          const int img = (int)(pix / ghw), rem = (int)(pix - (long)img * ghw);
          const int gy = rem / p.GW, gx = rem - gy * p.GW;
          const int sy = gy * p.SY + bdy, sx = gx * p.SX + bdx;
          if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W) vb[e] = X[(((long)img * p.H + sy) * p.W + sx) * p.Cs + bc];
        }
      }
    }
    if (p.bias_slab && tn == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bias_acc += va[e];  // this thread's column, pixels in order
    }
    __syncthreads();  // previous tile fully consumed
    {
      bf16x8 h, l;
      split8(va, h, l);
      *reinterpret_cast<bf16x8*>(&Ah[tcol * XP + tk * 8]) = h;
      *reinterpret_cast<bf16x8*>(&Al[tcol * XP + tk * 8]) = l;
      split8(vb, h, l);
      *reinterpret_cast<bf16x8*>(&Bh[tcol * XP + tk * 8]) = h;
      *reinterpret_cast<bf16x8*>(&Bl[tcol * XP + tk * 8]) = l;
    }
    __syncthreads();
    const int g = lane >> 4;
    bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = (wm * 32 + i * 16 + (lane & 15)) * XP + g * 8;
      ah[i] = *reinterpret_cast<const bf16x8*>(&Ah[o]);
      al[i] = *reinterpret_cast<const bf16x8*>(&Al[o]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o = (wn * 32 + j * 16 + (lane & 15)) * XP + g * 8;
      bh[j] = *reinterpret_cast<const bf16x8*>(&Bh[o]);
      bl[j] = *reinterpret_cast<const bf16x8*>(&Bl[o]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma3(ah[i], al[i], bh[j], bl[j], acc[i][j]);
  }
  float* out = p.slab + (long)split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (row < p.M && col < p.N) out[(long)row * p.N + col] = acc[i][j][r];
      }
    }
  if (p.bias_slab && tn == 0) {
    // fixed-order sum of the 4 k-group partials of each column (LDS, after the last tile)
    __shared__ float bred[4][FBM];
    bred[tk][tcol] = bias_acc;
    __syncthreads();
    if (tid < FBM && m0 + tid < p.M)
      p.bias_slab[(long)split * p.M + m0 + tid] = (bred[0][tid] + bred[1][tid]) + (bred[2][tid] + bred[3][tid]);
  }
}

static bool f32_split() {
  if (g_f32_mode < 0) g_f32_mode = 0;
  return g_f32_mode == 1;
}

void set_f32_mode(int mode) { g_f32_mode = mode ? 1 : 0; }
int get_f32_mode() { return f32_split() ? 1 : 0; }

// exact-f32 forward / dgrad tile: 128 x 128 (32x32x2 MFMA) while that still gives >= 1.5
// workgroups per CU, else 128 x 64 (the same kernel, one 32-column MFMA tile per wave) while that
// does, else the 64 x 64 16x16x4 kernel. (PMC, ResNet-9 b128: matrix-pipe busy 47.8% on the
// 128-row tiles vs 37.9% on the 64 x 64 kernel, profiles/pmc_f32_r4.md)
static int g2f_bn(int M, int N) {
  const long rows = (M + 127) / 128;
  if (N >= 128 && rows * ((N + 127) / 128) >= 384) return 128;
  if (N >= 64 && rows * ((N + 63) / 64) >= 384) return 64;
  return 0;  // the 64 x 64 kernel
}
static int g2f_bm(int M, int N) { return g2f_bn(M, N) ? 128 : FBM; }

void gemm_g2f(const G2Args& a, hipStream_t s) {
  if (a.ntaps > 64) throw std::runtime_error("gemm_g2f: at most 64 taps");
  const int bn = f32_split() ? 0 : g2f_bn(a.M, a.N);
  if (f32_split()) {
    const int tiles = ((a.M + FBM - 1) / FBM) * ((a.N + FBN - 1) / FBN);
    hipLaunchKernelGGL(gemm_g2x_kernel, dim3(tiles), dim3(256), 0, s, a);
  } else if (bn == 128) {
    const int tiles = ((a.M + 127) / 128) * ((a.N + 127) / 128);
    hipLaunchKernelGGL((gemm_g2f_wide_kernel<128, 128>), dim3(tiles), dim3(256), 0, s, a);
  } else if (bn == 64) {
    const int tiles = ((a.M + 127) / 128) * ((a.N + 63) / 64);
    hipLaunchKernelGGL((gemm_g2f_wide_kernel<128, 64>), dim3(tiles), dim3(256), 0, s, a);
  } else {
    const int tiles = ((a.M + FBM - 1) / FBM) * ((a.N + FBN - 1) / FBN);
    hipLaunchKernelGGL(gemm_g2f_kernel, dim3(tiles), dim3(256), 0, s, a);
  }
  DCNN_LAUNCH_CHECK();
}

int gemm_g2f_stat_rows(int M, int N) {
  const int bm = f32_split() ? FBM : g2f_bm(M, N);
  return (M + bm - 1) / bm;
}

// exact-f32 weight-gradient tile on the pixel-major 32x32x2 kernel: 128 rows / columns where the
// side holds at least 128, else 64 (fewer, larger split-K slabs: every split still gets one
// workgroup per CU or more). (PMC, ResNet-9 b128: matrix-pipe busy 43.1% on it vs 7.1% on the
// 64 x 64 16x16x4 kernel)
static void t2f_tile(int M, int N, int* bm, int* bn) {
  *bm = M >= 128 ? 128 : 64;
  *bn = N >= 128 ? 128 : 64;
}

int gemm_t2f_splits(int M, int N, int P) {
  int bm = FBM, bn = FBN;
  if (!f32_split()) t2f_tile(M, N, &bm, &bn);
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int splits = ((bm * bn >= 128 * 128 ? 512 : 1024) + tiles - 1) / tiles;
  const long max_by_k = (P + 255) / 256;             // at least 256 pixels per split
  if (splits > max_by_k) splits = (int)max_by_k;
  const long slab_cap = (96l << 20) / (4l * M * N);  // <= 96 MB of fp32 partials
  if (splits > slab_cap) splits = (int)(slab_cap > 0 ? slab_cap : 1);
  if (splits > 256) splits = 256;
  return splits < 1 ? 1 : splits;
}

void gemm_t2f(T2Args a, int splits, hipStream_t s) {
  if (a.ntaps > 64) throw std::runtime_error("gemm_t2f: at most 64 taps");
  const long per = (a.P + splits - 1) / splits;
  const int bk = f32_split() ? XBK : FBK;
  a.k_per_split = (int)(((per + bk - 1) / bk) * bk);
  if (f32_split()) {
    const int tiles = ((a.M + FBM - 1) / FBM) * ((a.N + FBN - 1) / FBN);
    hipLaunchKernelGGL(gemm_t2x_kernel, dim3(tiles * splits), dim3(256), 0, s, a);
  } else {
    int bm, bn;
    t2f_tile(a.M, a.N, &bm, &bn);
    const int tiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    if (bm == 128 && bn == 128)
      hipLaunchKernelGGL((gemm_t2f_wide_kernel<128, 128>), dim3(tiles * splits), dim3(256), 0, s, a);
    else if (bm == 128)
      hipLaunchKernelGGL((gemm_t2f_wide_kernel<128, 64>), dim3(tiles * splits), dim3(256), 0, s, a);
    else if (bn == 128)
      hipLaunchKernelGGL((gemm_t2f_wide_kernel<64, 128>), dim3(tiles * splits), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_t2f_wide_kernel<64, 64>), dim3(tiles * splits), dim3(256), 0, s, a);
  }
  DCNN_LAUNCH_CHECK();
}

// [Co][T][Ci] fp32 -> [Ci][T][Co] fp32 (dgrad B operand of the fp32 path)
__global__ void conv_weight_transpose_f32_kernel(const float* __restrict__ w, float* __restrict__ wt, int Co, int T,
                                                 int Ci) {
  const long n = (long)Co * T * Ci;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Co);
    const long r = i / Co;
    const int t = (int)(r % T), ci = (int)(r / T);
    wt[i] = w[((long)co * T + t) * Ci + ci];
  }
}

void conv_weight_transpose_f32(const float* w, float* wt, int Co, int T, int Ci, hipStream_t s) {
  const long n = (long)Co * T * Ci;
  const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(conv_weight_transpose_f32_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, w, wt, Co, T, Ci);
}

}  // namespace dcnn
