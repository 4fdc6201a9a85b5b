// RGB stem convolution (3x3, stride 1, pad 1, Ci <= 4, Co = 16..64) straight from the
// network's fp32 NCHW input, forward and weight gradient, on CDNA4 MFMA 16x16x32 bf16.
//
// The generic implicit GEMM (gemm2.hip) needs the input as NHWC bf16 with >= 8 channels, so the
// stem used to pay a layout/pad pass (nchw_to_nhwc_pad) and then ran a K = 72 GEMM whose
// 16-byte gathers carry 3 useful channels of 8 (~25 TFLOP/s, 7x over its memory floor). Here a
// workgroup owns a band of TH full image rows (TH * W = 512 output pixels) and stages its halo
// [(TH+2)][(W+2)][4 ch] once in LDS as bf16, converting from fp32 NCHW on the way in. The GEMM
// K axis is ordered (tap, channel-of-4): the 16x16x32 A fragment of a lane is two adjacent taps
// of one pixel = two 8-byte LDS reads, so K = 9 x 4 = 36 is two MFMA k-steps (taps 0-7, tap 8).
//
//   fwd:   y[p][co] = sum_k im2col(x)[p][k] * w[co][k]  (+ bias), bf16 NHWC, BN partial stats
//   wgrad: dW[co][k] = sum_p dY[p][co] * im2col(x)[p][k] ; column k = 36 of the B operand is
//          all ones, so the same MFMAs also produce the bias gradient sum_p dY[p][co].
//          Per-workgroup partials go to an fp32 slab reduced by splitk_reduce2.
#include "common.h"
#include "api.h"

namespace dcnn {

namespace {
constexpr int SPX = 512;          // output pixels per tile (TH * W)
constexpr int HALO_MAX = 6 * 130 * 4;  // bf16 elements of the forward halo (W <= 128)

__device__ __forceinline__ int stem_tiles(const StemArgs& p) { return p.N * (p.H / p.TH); }

// halo [(TH+2)][(W+2)][4] bf16 (8 bytes per pixel) of tile `tile` from fp32 NCHW, zero padded.
// Tiles span whole rows, so the left/right halo columns are always padding: the interior is
// read with 16-byte loads (4 pixels of one channel row, all of a thread's loads issued before
// its first LDS store), and the padding columns / channels >= Ci are zero-filled. The three
// sets are disjoint: no ordering between them is needed.
__device__ __forceinline__ void stage_halo(const StemArgs& p, int tile, bf16* hs) {
  constexpr int J = 3;  // interior float4 per thread: Ci * (TH+2) * W/4 <= 768 (stem_supported)
  const int tpi = p.H / p.TH, n = tile / tpi, y0 = (tile - n * tpi) * p.TH;
  const int HW2 = p.W + 2, rows = p.TH + 2, w4 = p.W >> 2, per_c = rows * w4, total = p.Ci * per_c;
  float4 v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int i = threadIdx.x + j * 256;
    const int c = i / per_c, r = i - c * per_c, hy = r / w4, x4 = r - hy * w4;
    const int y = y0 + hy - 1;
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < total && (unsigned)y < (unsigned)p.H)
      v[j] = *reinterpret_cast<const float4*>(p.x + (((long)n * p.Ci + c) * p.H + y) * p.W + x4 * 4);
  }
  for (int i = threadIdx.x; i < (4 - p.Ci) * rows * HW2; i += 256) {  // channels >= Ci
    const int c = p.Ci + i / (rows * HW2), r = i % (rows * HW2);
    hs[r * 4 + c] = (bf16)0.f;
  }
  for (int i = threadIdx.x; i < p.Ci * rows * 2; i += 256) {  // left / right padding columns
    const int c = i / (rows * 2), r = i % (rows * 2), hy = r >> 1;
    hs[(hy * HW2 + (r & 1) * (HW2 - 1)) * 4 + c] = (bf16)0.f;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int i = threadIdx.x + j * 256;
    const int c = i / per_c, r = i - c * per_c, hy = r / w4, x4 = r - hy * w4;
    if (i < total) {
      bf16* d = hs + (hy * HW2 + 1 + x4 * 4) * 4 + c;
      d[0] = (bf16)v[j].x; d[4] = (bf16)v[j].y; d[8] = (bf16)v[j].z; d[12] = (bf16)v[j].w;
    }
  }
}

__device__ __forceinline__ float wval(const StemArgs& p, int co, int tap, int ch) {
  if (ch >= p.Ci || tap > 8) return 0.f;
  const long o = co * p.ws[0] + ch * p.ws[1] + (tap / 3) * p.ws[2] + (tap % 3) * p.ws[3];
  return p.w_bf16 ? (float)reinterpret_cast<const bf16*>(p.w)[o] : reinterpret_cast<const float*>(p.w)[o];
}

__device__ __forceinline__ bf16x8 cat44(bf16x4 lo, bf16x4 hi) {
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
}  // namespace

// ---------------------------------------------------------------------------------------------
// forward: one tile per workgroup, wave w takes 16-pixel groups w, w+4, ...
// ---------------------------------------------------------------------------------------------
template <int NCB>
// <= 64 VGPRs for Co <= 32: 8 workgroups per CU, a ResNet stem's whole grid resident at once
__global__ void __launch_bounds__(256, NCB <= 2 ? 8 : 4) stem_fwd_kernel(StemArgs p) {
  constexpr int CO = NCB * 16;
  __shared__ __attribute__((aligned(16))) bf16 halo[HALO_MAX];
  __shared__ __attribute__((aligned(16))) bf16 stg[4][16 * CO];
  __shared__ float red[4][3][CO];  // per wave: pivot-shifted (sum, sum^2) and the pivot
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, kg = lane >> 4, col = lane & 15;
  const int tile = blockIdx.x;
  if (p.zero_ptr && tile == 0)
    for (int i = threadIdx.x; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;
  stage_halo(p, tile, halo);

  // B fragments (weights), k-step 0: taps 2kg, 2kg+1; k-step 1: tap 8 in lane group 0
  bf16x8 b0[NCB], b1[NCB];
  float bias[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int co = cb * 16 + col;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b0[cb][e] = (bf16)wval(p, co, 2 * kg + (e >> 2), e & 3);
      b1[cb][e] = (bf16)(kg == 0 ? wval(p, co, 8, e & 3) * (e < 4) : 0.f);
    }
    bias[cb] = p.bias ? p.bias[co] : 0.f;
  }
  __syncthreads();

  const int HW2 = p.W + 2;
  const int tpi = p.H / p.TH, n = tile / tpi, y0 = (tile - n * tpi) * p.TH;
  // per-lane tap offsets (in halo pixels) of the A fragment: taps 2kg, 2kg+1 and tap 8
  const int t0 = 2 * kg, t1 = 2 * kg + 1;
  const int o0 = (t0 / 3) * HW2 + t0 % 3, o1 = (t1 / 3) * HW2 + t1 % 3, o8 = 2 * HW2 + 2;
  // statistics are summed about a per-wave pivot (the wave's first output row of each channel)
  // and merged over the 4 waves with Chan's update: (count, mean, M2) triples, fixed order
  float s[NCB], q[NCB], piv[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) s[cb] = q[cb] = piv[cb] = 0.f;
  bool first = true;
  const bf16x4 z4 = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
  for (int g = wid; g < SPX / 16; g += 4) {
    const int px = g * 16 + col, py = px / p.W, pxx = px - py * p.W;
    const int hp = py * HW2 + pxx;  // halo pixel of tap (0, 0)
    const bf16x4* h4 = reinterpret_cast<const bf16x4*>(halo);
    const bf16x8 a0 = cat44(h4[hp + o0], h4[hp + o1]);
    const bf16x8 a1 = cat44(kg == 0 ? h4[hp + o8] : z4, z4);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[cb], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[cb], acc, 0, 0, 0);
      if (first) piv[cb] = __shfl((float)(bf16)(acc[0] + bias[cb]), col, 64);  // row 0 of this column
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bf16 v = (bf16)(acc[r] + bias[cb]);
        const float f = (float)v - piv[cb];
        s[cb] += f;
        q[cb] += f * f;
        stg[wid][(kg * 4 + r) * CO + cb * 16 + col] = v;
      }
    }
    first = false;
    // the 16 pixels of a group are contiguous in NHWC: 16 * CO * 2 bytes, 16 per lane
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const long obase = (((long)n * p.H + y0) * p.W + g * 16) * CO;
    for (int c = lane; c < 2 * CO; c += 64)
      reinterpret_cast<uint4*>(p.y + obase)[c] = reinterpret_cast<const uint4*>(stg[wid])[c];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (!p.slab) return;
  // channel sums: lane groups (kg) via cross-lane adds, then the 4 waves through LDS
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    s[cb] += __shfl_xor(s[cb], 16);
    s[cb] += __shfl_xor(s[cb], 32);
    q[cb] += __shfl_xor(q[cb], 16);
    q[cb] += __shfl_xor(q[cb], 32);
    if (kg == 0) {
      red[wid][0][cb * 16 + col] = s[cb];
      red[wid][1][cb * 16 + col] = q[cb];
      red[wid][2][cb * 16 + col] = piv[cb];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < CO; c += 256) {
    Welford t{0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int ng = w < SPX / 16 ? (SPX / 16 - 1 - w) / 4 + 1 : 0;  // groups this wave ran
      t = welford_merge(t, welford_from_shifted((float)(ng * 16), red[w][2][c], red[w][0][c], red[w][1][c]));
    }
    store_welford(p.slab, tile, CO, c, t);
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient: workgroup b accumulates tiles b, b + grid, ...; each tile's 16 k-steps of 32
// pixels are split over the 4 waves. D[co][k] with k = tap*4 + ch (k < 36), k = 36: ones.
// ---------------------------------------------------------------------------------------------
// BNT: the BatchNorm-backward transform of dy (StemArgs::bn_x; the stem BatchNorm's data gradient
// is never written: this kernel is its only consumer). The 16-byte vectors of each staged dY tile
// are rewritten in LDS as bf16(A dy + B (x - mean) + D), the exact arithmetic and rounding of
// bn_bwd_apply_v_kernel, so the weight gradient is bit-identical to the unfused pair of passes.
template <int NCB, bool BNT>
__global__ void __launch_bounds__(256, NCB <= 2 ? (BNT ? 3 : 4) : 2) stem_wgrad_kernel(StemArgs p) {
  constexpr int CO = NCB * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = reinterpret_cast<bf16*>(smem);                     // [(TH+2)(W+2)][4]
  bf16* dys = reinterpret_cast<bf16*>(smem + p.halo_bytes);       // [512][CO]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, kg = lane >> 4, col = lane & 15;
  const int HW2 = p.W + 2;
  const int ntile = stem_tiles(p);
  const i32x4 rs_dy = raw_rsrc(p.dy, (unsigned)((long)p.N * p.H * p.W * CO * 2));
  // [4][CO] after the dY tile: A, B, mean, D (BNT)
  float* coef = reinterpret_cast<float*>(smem + p.halo_bytes + SPX * CO * 2);
  if constexpr (BNT) {
    for (int c = threadIdx.x; c < CO; c += 256) {
      // the reduced sums as bn_bwd_apply_v_kernel reads them (read_stats<1>: parts merged in order)
      float sdy, sdyx;
      if (p.bn_parts <= 1) {
        sdy = p.bn_sums[c];
        sdyx = p.bn_sums[CO + c];
      } else {
        sdy = p.bn_sums[c];
        sdyx = p.bn_sums[CO + c];
        for (int q = 1; q < p.bn_parts; ++q) {
          sdy += p.bn_sums[(long)q * 3 * CO + c];
          sdyx += p.bn_sums[(long)q * 3 * CO + CO + c];
        }
      }
      const float is = p.bn_istd[c], a = (p.bn_gamma ? p.bn_gamma[c] : 1.f) * is;
      coef[c] = a;
      coef[CO + c] = p.bn_eval ? 0.f : -a * is * (sdyx / p.bn_count);
      coef[2 * CO + c] = p.bn_mean[c];
      coef[3 * CO + c] = p.bn_eval ? 0.f : -a * (sdy / p.bn_count);
      if (blockIdx.x == 0) {
        if (p.bn_dgamma) p.bn_dgamma[c] += sdyx;
        if (p.bn_dbeta) p.bn_dbeta[c] += sdy;
      }
    }
  }
  constexpr int NVT = SPX * CO / 8 / 256;  // 16-byte vectors of a dY tile per thread
  f32x4 acc[NCB][3];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) acc[cb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B column of this lane in each of the 3 n-blocks: k = nb*16 + col -> (tap, ch); k = 36: ones
  int koff[3];
  bool kval[3], kone[3];
#pragma unroll
  for (int nb = 0; nb < 3; ++nb) {
    const int k = nb * 16 + col, tap = k >> 2, ch = k & 3;
    kval[nb] = k < 36 && ch < p.Ci;
    kone[nb] = k == 36;
    koff[nb] = ((tap < 9 ? (tap / 3) * HW2 + tap % 3 : 0) * 4) + ch;
  }
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    __syncthreads();  // previous tile's fragments consumed
    const int tpi = p.H / p.TH, n = tile / tpi, y0 = (tile - n * tpi) * p.TH;
    // the dY tile is contiguous in NHWC: 16-byte direct-to-LDS loads, 1 KB per wave instruction
    const unsigned src = (unsigned)((((long)n * p.H + y0) * p.W) * CO * 2);
#pragma unroll
    for (int j = 0; j < SPX * CO * 2 / 1024 / 4; ++j) {
      const int blk = wid * (SPX * CO * 2 / 1024 / 4) + j;
      glds16_opaque(rs_dy, reinterpret_cast<char*>(dys) + blk * 1024, src + blk * 1024 + lane * 16);
    }
    stage_halo(p, tile, halo);
    // the BatchNorm input rows of the tile (same NHWC offsets as dY), issued before the wait for
    // the dY tile so their latency overlaps it (BNT instances run 3 workgroups per CU: the 4-per-CU
    // register budget spills with these in flight)
    uint4 xv[BNT ? NVT : 1];
    if constexpr (BNT) {
      const char* xb = reinterpret_cast<const char*>(p.bn_x) + src;
#pragma unroll
      for (int j = 0; j < NVT; ++j) xv[j] = *reinterpret_cast<const uint4*>(xb + (threadIdx.x + j * 256) * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (BNT) {
      {
        constexpr int j0 = 0, RV = NVT;
#pragma unroll
        for (int j = 0; j < RV; ++j) {
          const int v = threadIdx.x + (j0 + j) * 256;
          int c0 = (v % (CO / 8)) * 8;
          // (opaque per round: keeps the coefficient reads here instead of hoisted out of the tile
          // loop, where 32 more live registers would spill across the MFMA loop)
          asm volatile("" : "+v"(c0));
          uint4* q = reinterpret_cast<uint4*>(dys) + v;
          float d[8], xf[8];
          unpack8(*q, d);
          unpack8(xv[j], xf);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            d[e] = coef[c0 + e] * d[e] + coef[CO + c0 + e] * (xf[e] - coef[2 * CO + c0 + e]) + coef[3 * CO + c0 + e];
          *q = pack8(d);
        }
      }
      __syncthreads();
    }
    for (int ks = wid; ks < SPX / 32; ks += 4) {
      // this lane's 8 pixels (GEMM k) of the step: ks*32 + kg*8 .. +7, all in one image row
      const int p0 = ks * 32 + kg * 8, py = p0 / p.W, px0 = p0 - py * p.W;
      bf16x8 a[NCB], b[3];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int e = 0; e < 8; ++e) a[cb][e] = dys[(p0 + e) * CO + cb * 16 + col];
      const int hb = (py * HW2 + px0) * 4;
#pragma unroll
      for (int nb = 0; nb < 3; ++nb)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          b[nb][e] = kval[nb] ? halo[hb + e * 4 + koff[nb]] : (bf16)(kone[nb] ? 1.f : 0.f);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) acc[cb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cb], b[nb], acc[cb][nb], 0, 0, 0);
    }
  }
  // 4 waves -> one partial: D rows (co) = 4*kg + r of block cb, column k = nb*16 + col
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4][CO][48]
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int nb = 0; nb < 3; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wid * CO + cb * 16 + kg * 4 + r) * 48 + nb * 16 + col] = acc[cb][nb][r];
  __syncthreads();
  float* out = p.slab + (long)blockIdx.x * p.n_slab;
  for (int i = threadIdx.x; i < CO * 37; i += 256) {
    const int co = i / 37, k = i - co * 37, tap = k >> 2, ch = k & 3;
    const float v = red[(0 * CO + co) * 48 + k] + red[(1 * CO + co) * 48 + k] + red[(2 * CO + co) * 48 + k] +
                    red[(3 * CO + co) * 48 + k];
    if (k == 36) {
      if (p.bias_slab) p.bias_slab[(long)blockIdx.x * CO + co] = v;
    } else if (ch < p.Ci) {
      out[co * p.gs[0] + ch * p.gs[1] + (tap / 3) * p.gs[2] + (tap % 3) * p.gs[3]] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
bool stem_supported(int N, int Ci, int H, int W, int Co) {
  if (Ci < 1 || Ci > 4 || Co % 16 || Co > 64 || W % 16 || SPX % W) return false;
  const int th = SPX / W;
  if (H % th || (th + 2) * (W + 2) * 4 > HALO_MAX || Ci * (th + 2) * (W / 4) > 3 * 256) return false;
  return N > 0 && (long)N * Ci * H * W < (1l << 31);
}

int stem_tiles_host(int N, int H, int W) { return N * (H / (SPX / W)); }

int stem_wgrad_blocks(int N, int H, int W) {
  const int t = stem_tiles_host(N, H, W);
  return t < 1024 ? t : 1024;
}

// the BatchNorm-folding instance holds 3 workgroups per CU (its register budget): one resident
// wave of workgroups instead of 1024 (DCNN_STEM_BNT_BLOCKS: experiment override)
int stem_wgrad_blocks_bnt(int N, int H, int W) {
  static const int forced = [] {
    const char* e = std::getenv("DCNN_STEM_BNT_BLOCKS");
    return e ? std::atoi(e) : 0;
  }();
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int t = stem_tiles_host(N, H, W), want = forced > 0 ? forced : 3 * cus;
  return t < want ? t : want;
}

void stem_fwd(StemArgs a, hipStream_t s) {
  if (!stem_supported(a.N, a.Ci, a.H, a.W, a.Co)) throw std::runtime_error("stem_fwd: unsupported shape");
  a.TH = SPX / a.W;
  const int grid = stem_tiles_host(a.N, a.H, a.W);
  switch (a.Co / 16) {
    case 1: hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(grid), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3(grid), dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(stem_fwd_kernel<3>, dim3(grid), dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(stem_fwd_kernel<4>, dim3(grid), dim3(256), 0, s, a); break;
  }
  DCNN_LAUNCH_CHECK();
}

void stem_wgrad(StemArgs a, int blocks, hipStream_t s) {
  if (!stem_supported(a.N, a.Ci, a.H, a.W, a.Co)) throw std::runtime_error("stem_wgrad: unsupported shape");
  if (blocks < 1 || blocks > stem_tiles_host(a.N, a.H, a.W)) throw std::runtime_error("stem_wgrad: bad block count");
  a.TH = SPX / a.W;
  a.halo_bytes = (((a.TH + 2) * (a.W + 2) * 8) + 15) / 16 * 16;
  const bool bnt = a.bn_x != nullptr;
  if (bnt && (!a.bn_mean || !a.bn_istd || !a.bn_sums || a.bn_parts < 1 || a.bn_count <= 0.f))
    throw std::runtime_error("stem_wgrad: incomplete BatchNorm-backward operands");
  const int main = a.halo_bytes + SPX * a.Co * 2 + (bnt ? 4 * a.Co * 4 : 0), epi = 4 * a.Co * 48 * 4;
  const int lds = main > epi ? main : epi;
#define DCNN_SW(C)                                                                                        \
  {                                                                                                       \
    auto k = bnt ? stem_wgrad_kernel<C, true> : stem_wgrad_kernel<C, false>;                              \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, s, a);                                            \
  }
  switch (a.Co / 16) {
    case 1: DCNN_SW(1) break;
    case 2: DCNN_SW(2) break;
    case 3: DCNN_SW(3) break;
    default: DCNN_SW(4) break;
  }
#undef DCNN_SW
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
