// Streaming 1x1 convolution (and its stride-1 data gradient) for CDNA4: wave-independent,
// weight-stationary, no barriers in the tile loop.
//
// Why (profiles/conv_r50_r3.md): the 1x1 convs of a ResNet bottleneck have K = 64..128 input
// channels, so the gathered GEMM (gemm2.hip) runs ONE K step per 128x128 tile and then a
// two-barrier LDS epilogue; each workgroup is a latency chain (load -> 32 MFMAs -> LDS round trip
// -> stores + statistics) and the expand convs (64 -> 256 at 32x32, batch 256) ran at 1.6 TB/s,
// 5x off their HBM floor.
//
// Here every wave is its own pipeline:
//  * a wave owns 64 output channels (the A operand) and a contiguous range of 32-pixel tiles.
//    K = 64 / 128: its weights [64][K] live in VGPRs for the whole kernel (loaded once);
//    K = 256 / 512 (and the K = 128 data gradient): the workgroup's 4 waves share one channel slice
//    whose weights sit in LDS (rows padded by 16 B: conflict-free, immediate-offset fragment
//    reads), and B streams in 128-channel chunks through a two-buffer register ring;
//  * per tile it loads the B fragments (16 pixels x 8 channels per lane, 16-byte global loads
//    straight into registers, the next tile's issued before this tile's MFMAs), issues
//    16 x K/32 mfma_f32_16x16x32_bf16 per 64 channels, and runs the epilogue from registers: an
//    accumulator quad is 4 consecutive channels of one pixel, staged in the wave's LDS slice and
//    stored as full 128-byte pixel rows (8 lanes per row);
//  * BatchNorm statistics accumulate in registers across all tiles of the wave (pivot-shifted
//    sums, packed fp32 math) and are reduced over the 16 lanes of a DPP row ONCE per wave, so the
//    statistics slab has one row per pixel range instead of one per 128-pixel tile (the
//    bn_stat_reduce that follows reads 8-16x fewer rows);
//  * no barriers after the prologue: the waves of a CU drift into different phases, so one
//    wave's epilogue VALU and stores overlap another's MFMAs and loads.
//
// Modes: 0 plain (optional bias / residual / ReLU), 1 forward with Welford statistics of the
// stored values, 2 data gradient with the backward-BatchNorm fusion of the producing layer
// (ReLU mask from its output y, sums of g and g * xhat: the same contract as gemm_g2's bnb
// epilogue, api.h BnbArgs).
//
// Reference parity: the reference runs 1x1 convs through im2col + cuBLAS / cuDNN
// (src/nn/layers_impl/cuda/conv2d_ops.cu:18-128, cudnn_conv2d_ops.cu:187-244).
#include <array>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "api.h"

namespace dcnn {

namespace {
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int xcd_remap_g1(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// fixed-order sum over the 16 lanes of a DPP row; every lane of the row gets the total
__device__ __forceinline__ float g1_row_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad xor 2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad xor 1
  return v;
}

// value held by lane 0 of this lane's 16-lane row
__device__ __forceinline__ float g1_row_first(float v) {
  // DPP row_newbcast:0 (gfx90a+): lane 0 of each 16-lane row to the whole row, one instruction
  // (four readlanes + selects before)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150, 0xf, 0xf, false));
}

// two bf16 of one 32-bit word -> fp32 pair (exact)
__device__ __forceinline__ f32x2 bf2_to_f2(unsigned w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ unsigned f2_to_bf2(float a, float b) {
  bf16 x = (bf16)a, y = (bf16)b;
  return (unsigned)__builtin_bit_cast(unsigned short, x) | ((unsigned)__builtin_bit_cast(unsigned short, y) << 16);
}
}  // namespace

struct G1sArgs {
  const bf16* X; const bf16* Wt; bf16* Y;
  int M, N, K, H, W, OH, OW, S;  // output pixels M = NB * OH * OW, input NB x H x W x K (NHWC)
  int PR, tpr, tiles;            // pixel ranges (statistics rows), tiles per range, M / tile pixels
  const float* bias; const bf16* residual; float* stats; int relu;
  float* zero_ptr; int zero_n;
  BnbArgs bnb;
  int gen, ntaps, Kc, ldw, GH, GW, OS, ORY, ORX, OHo, OWo;
  int tap_dy[4], tap_dx[4], tap_k[4];
};

// per-instance shape: TJ 16-pixel subtiles per tile, OCC waves per SIMD the registers allow
// (K = 64: 32-pixel tiles keep the forward at ~150 VGPRs, three waves per SIMD to hide the
// load latency behind each other's epilogues)
// target waves per SIMD of the pixel-range split (tuning hook; profiles/split_target_r4.md)
static int g_g1s_wps = 2;
void g1s_set_waves_per_simd(int w) { g_g1s_wps = w < 1 ? 1 : w; }
static int g1s_occ_rt(int K, int mode) { (void)K; (void)mode; return g_g1s_wps; }  // waves per SIMD
// (K = 32: one MFMA k step per subtile; weights 16 VGPRs)
constexpr int kG1sTile = 32;  // pixels per tile (16 * TJ)
// weights in LDS (shared by the workgroup's 4 waves) instead of VGPRs: K >= 256, and the K = 128
// data gradient (its three epilogue operands leave no room for 64 weight VGPRs)
constexpr bool g1s_wl(int K, int mode) { return K >= 256 || (K == 128 && mode == 2); }

template <int K, int MODE, int OCC, int PF, bool EP, bool GEN = false>
__global__ void __launch_bounds__(256, OCC) g1s_kernel(G1sArgs p) {
  prefetch_kernargs<sizeof(G1sArgs)>();
  constexpr int KK = K / 32, TJ = 2, TP = 16 * TJ;
  // K >= 256: the 64 x K weight slice lives in LDS, shared by the workgroup's 4 waves (same
  // channel slice, 4 pixel ranges), instead of K / 2 VGPRs per lane
  constexpr bool WL = g1s_wl(K, MODE);
  // output stage only where the LDS budget keeps two workgroups per CU
  constexpr bool STG = K <= 256;
  static_assert(TP == kG1sTile, "tile size");
  static_assert(PF == 1 || PF == 2 || PF == 4, "prefetch depth (the tile loop is unrolled by it)");
  static_assert(PF == 2 || !EP, "epilogue-operand ping-pong assumes the 2-tile unroll");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  // per-wave channel constants (bias or BatchNorm mean / 1/std, and the statistics pivots of this
  // wave's 64 channels) and the per-wave output stage; each wave touches only its own slices
  // (no barrier: LDS ops of one wave execute in order, and LDS reads never wait for stores)
  __shared__ __attribute__((aligned(16))) float cst[4][2][64];
  __shared__ __attribute__((aligned(16))) char stage[4][STG ? TP * 128 : 16];
  constexpr int WPITCH = K * 2 + 16;
  __shared__ __attribute__((aligned(16))) char wlds[WL ? 64 * WPITCH : 16];
  char* stg = stage[wid];
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = threadIdx.x; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;
  const int CS = p.N >> 6;
  const int blk = xcd_remap_g1(blockIdx.x, gridDim.x);
  // weight-row column of GEMM channel k (k .. k + 7 stay inside one tap: Kc % 32 == 0)
  auto wcol = [&](int k) { return p.tap_k[k / p.Kc] + k % p.Kc; };
  int cs, pr;
  if (WL) {  // workgroup = one channel slice x 4 consecutive pixel ranges
    cs = blk % CS;
    pr = (blk / CS) * 4 + wid;
    // rows padded by one 16-byte chunk (pitch WPITCH): the 16 rows an A-fragment read group
    // touches start on 16 distinct bank slots (conflict-free ds_read_b128), and every fragment
    // address is one per-lane base plus an immediate
    for (int q = threadIdx.x; q < 64 * (K / 8); q += 256) {
      const int r = q / (K / 8), c = q % (K / 8);
      *reinterpret_cast<uint4*>(wlds + r * WPITCH + c * 16) =
          *reinterpret_cast<const uint4*>(p.Wt + (size_t)(cs * 64 + r) * p.ldw + wcol(c * 8));
    }
    __syncthreads();
  } else {
    const int gw = blk * 4 + wid;
    if (gw >= p.PR * CS) return;
    cs = gw % CS;
    pr = gw / CS;
  }
  const int n0 = cs * 64;
  const int t0 = min(p.tiles, pr * p.tpr), t1 = min(p.tiles, t0 + p.tpr);

  if (MODE == 2) {
    cst[wid][0][lane] = p.bnb.mean[n0 + lane];
    cst[wid][1][lane] = p.bnb.istd[n0 + lane];
  } else {
    cst[wid][0][lane] = p.bias ? p.bias[n0 + lane] : 0.f;
  }
  // weights: A fragment (channel subtile i, k step kk): row n0 + 16 i + lr, k = 32 kk + 8 lh
  bf16x8 wa[4][WL ? 1 : KK];
  if constexpr (!WL) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        wa[i][kk] = *reinterpret_cast<const bf16x8*>(p.Wt + (size_t)(n0 + i * 16 + lr) * p.ldw + wcol(kk * 32 + lh * 8));
  }
  int wl_off = lr * WPITCH + lh * 16;
  auto afrag = [&](int i, int kk) -> bf16x8 {
    if constexpr (WL) {
      return *reinterpret_cast<const bf16x8*>(wlds + wl_off + i * 16 * WPITCH + kk * 64);
    } else {
      return wa[i][kk];
    }
  };

  const bool plain = !GEN && p.S == 1 && p.OH == p.H && p.OW == p.W;
  const int ohw = p.OH * p.OW, ghw = p.GH * p.GW;
  auto src_px = [&](int m) -> long {  // input pixel of output pixel m (gen = 0)
    if (plain) return m;
    const int img = m / ohw, rem = m - img * ohw;
    const int oy = rem / p.OW, ox = rem - oy * p.OW;
    return ((long)img * p.H + oy * p.S) * p.W + ox * p.S;
  };
  // gen = 1: element offset of (GEMM row m, channel k) in the input, or -1 outside the image
  auto src_gen = [&](int m, int k) -> long {
    const int img = m / ghw, rem = m - img * ghw;
    const int gy = rem / p.GW, gx = rem - gy * p.GW;
    const int t = k / p.Kc, c = k - t * p.Kc;
    const int sy = gy + p.tap_dy[t], sx = gx + p.tap_dx[t];
    if ((unsigned)sy >= (unsigned)p.H || (unsigned)sx >= (unsigned)p.W) return -1;
    return (((long)img * p.H + sy) * p.W + sx) * p.Kc + c;
  };
  // output pixel row of GEMM row m
  auto orow = [&](int m) -> long {
    if (!GEN) return m;
    const int img = m / ghw, rem = m - img * ghw;
    const int gy = rem / p.GW, gx = rem - gy * p.GW;
    return ((long)img * p.OHo + gy * p.OS + p.ORY) * p.OWo + gx * p.OS + p.ORX;
  };
  const bf16x8 zero8 = {};
  auto ldb8 = [&](int m, int k) -> bf16x8 {  // one B fragment, gathered form
    const long o = src_gen(m, k);
    return o >= 0 ? *reinterpret_cast<const bf16x8*>(p.X + o) : zero8;
  };
  // B fragments of PF tiles in flight (ring, statically indexed by the unrolled loop)
  bf16x8 bb[PF][TJ][WL ? 1 : KK];
  auto load_b = [&](bf16x8 (&b)[TJ][WL ? 1 : KK], int t) {
    if constexpr (WL) return;
    if (GEN) {
      if (p.ntaps == 0) return;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) b[j][kk] = ldb8(t * TP + j * 16 + lr, kk * 32 + lh * 8);
      return;
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const bf16* q = p.X + src_px(t * TP + j * 16 + lr) * K + lh * 8;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) b[j][kk] = *reinterpret_cast<const bf16x8*>(q + kk * 32);
    }
  };
  // epilogue operands (residual or the BatchNorm's y, and its x), one tile ahead (ping-pong)
  const bool has_res = MODE != 1 && p.residual != nullptr;
  const bool has_y = MODE == 2 && p.bnb.y != nullptr;
  const bool has_e = has_res || MODE == 2;
  const bool relu = MODE == 0 && p.relu;
  // e[0]: residual (modes 0 / 2), e[1]: the BatchNorm's x (mode 2), e[2]: its output y (mode 2)
  constexpr int NE = MODE == 2 ? 3 : 1;
  uint2 eo[2][NE][4][TJ];
  auto load_e = [&](uint2 (&e)[NE][4][TJ], int t) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const size_t row = (size_t)orow(t * TP + j * 16 + lr) * p.N + n0 + lh * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        e[0][i][j] = has_res ? *reinterpret_cast<const uint2*>(p.residual + row + i * 16) : make_uint2(0u, 0u);
        if constexpr (MODE == 2) {
          e[1][i][j] = *reinterpret_cast<const uint2*>(p.bnb.x + row + i * 16);
          e[2][i][j] = has_y ? *reinterpret_cast<const uint2*>(p.bnb.y + row + i * 16) : make_uint2(0u, 0u);
        }
      }
    }
  };

  // statistics accumulators: channel n0 + 16 i + 4 lh + r, summed over this lane's pixels
  f32x2 sa[4][2], sb[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) sa[i][h] = sb[i][h] = f32x2{0.f, 0.f};

  // one tile: the load of tile t + PF - 1 goes out first (into the buffer tile t - 1 used), then
  // the MFMAs, the next tile's epilogue operands, and the epilogue of this one
  // K >= 256: B streams in 128-channel chunks through a two-buffer ring (bq), the next tile's
  // first chunk loading during this tile's last chunk
  constexpr int NC = WL ? KK / 4 : 1;
  bf16x8 bq[2][TJ][4];
  auto load_chunk = [&](bf16x8 (&b)[TJ][4], int t, int c) {
    if (GEN) {
      if (p.ntaps == 0) return;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) b[j][u] = ldb8(t * TP + j * 16 + lr, c * 128 + u * 32 + lh * 8);
      return;
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const bf16* q = p.X + src_px(t * TP + j * 16 + lr) * K + c * 128 + lh * 8;
#pragma unroll
      for (int u = 0; u < 4; ++u) b[j][u] = *reinterpret_cast<const bf16x8*>(q + u * 32);
    }
  };
  auto tile = [&](int t, bf16x8 (&bc)[TJ][WL ? 1 : KK], bf16x8 (&bn)[TJ][WL ? 1 : KK], uint2 (&ec)[NE][4][TJ], uint2 (&en)[NE][4][TJ]) {
    f32x4 acc[4][TJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (GEN && p.ntaps == 0) {
      // a stride phase no tap reaches: the epilogue alone (residual or zero)
    } else if constexpr (WL) {
      // the weight slice never changes after the barrier: keep the compiler from hoisting all
      // 4 x K / 32 fragment reads out of the tile loop (K / 2 VGPRs of live fragments)
      asm volatile("" : "+v"(wl_off));
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        // the next tile's first chunk goes to the buffer its first chunk is read from, bq[0]:
        // with an even chunk count that is the other buffer, loaded during this tile's last
        // chunk; with one chunk (K = 128) it is the buffer being read, reloaded after the MFMAs
        // below (loading it into bq[1] left tile t + 1 computing on tile t's operands)
        if (c + 1 < NC) load_chunk(bq[(c + 1) & 1], t, c + 1);
        else if (NC % 2 == 0 && t + 1 < t1) load_chunk(bq[(c + 1) & 1], t + 1, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 av = afrag(i, c * 4 + u);
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bq[c & 1][j][u], acc[i][j], 0, 0, 0);
          }
      }
      static_assert(NC == 1 || NC % 2 == 0, "chunk ring parity");
      if (NC == 1 && t + 1 < t1) load_chunk(bq[0], t + 1, 0);
    } else {
      if (PF > 1 && t + PF - 1 < t1) load_b(bn, t + PF - 1);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x8 av = afrag(i, kk);
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bc[j][kk], acc[i][j], 0, 0, 0);
        }
      if (PF == 1 && t + 1 < t1) load_b(bc, t + 1);  // one buffer: reloaded once the MFMAs have read it
    }
    if (has_e) {
      if (EP) { if (t + 1 < t1) load_e(en, t + 1); }
      else load_e(ec, t);  // operand loads still ahead of this tile's stores
    }
    const bool first = t == t0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 c0 = *reinterpret_cast<const float4*>(&cst[wid][0][i * 16 + lh * 4]);
      if (MODE == 1 && first) {
        // statistics pivot of each channel: the stored value of the wave's first pixel
        const float v0 = (float)(bf16)(acc[i][0][0] + c0.x), v1 = (float)(bf16)(acc[i][0][1] + c0.y);
        const float v2 = (float)(bf16)(acc[i][0][2] + c0.z), v3 = (float)(bf16)(acc[i][0][3] + c0.w);
        const float p0 = g1_row_first(v0), p1 = g1_row_first(v1), p2 = g1_row_first(v2), p3 = g1_row_first(v3);
        if (lr == 0) *reinterpret_cast<float4*>(&cst[wid][1][i * 16 + lh * 4]) = make_float4(p0, p1, p2, p3);
      }
      const float4 c1 = MODE != 0 ? *reinterpret_cast<const float4*>(&cst[wid][1][i * 16 + lh * 4]) : c0;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        float f[4];
        if (MODE == 2) {
#pragma unroll
          for (int r = 0; r < 4; ++r) f[r] = acc[i][j][r];
        } else {
          f[0] = acc[i][j][0] + c0.x; f[1] = acc[i][j][1] + c0.y; f[2] = acc[i][j][2] + c0.z; f[3] = acc[i][j][3] + c0.w;
        }
        if (has_res) {
          const f32x2 r01 = bf2_to_f2(ec[0][i][j].x), r23 = bf2_to_f2(ec[0][i][j].y);
          f[0] += r01.x; f[1] += r01.y; f[2] += r23.x; f[3] += r23.y;
        }
        if (relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) f[r] = fmaxf(f[r], 0.f);
        }
        if (has_y) {
          const f32x2 y01 = bf2_to_f2(ec[NE - 1][i][j].x), y23 = bf2_to_f2(ec[NE - 1][i][j].y);
          f[0] = y01.x > 0.f ? f[0] : 0.f; f[1] = y01.y > 0.f ? f[1] : 0.f;
          f[2] = y23.x > 0.f ? f[2] : 0.f; f[3] = y23.y > 0.f ? f[3] : 0.f;
        }
        const uint2 o = make_uint2(f2_to_bf2(f[0], f[1]), f2_to_bf2(f[2], f[3]));
        if (!STG) {  // direct 8-byte stores (16 pixel rows x 32 B per instruction)
          *reinterpret_cast<uint2*>(p.Y + (size_t)orow(t * TP + j * 16 + lr) * p.N + n0 + lh * 4 + i * 16) = o;
        } else {
          // full-line stores: the tile's 32 pixel rows (128 B each, 16-byte chunks XOR-swizzled by
          // the pixel) are staged in this wave's LDS slice and read back as 8 lanes per pixel row
          const int P = j * 16 + lr, c = i * 2 + (lh >> 1);
          *reinterpret_cast<uint2*>(stg + P * 128 + ((c ^ (P & 7)) << 4) + (lh & 1) * 8) = o;
        }
        if constexpr (MODE == 1) {
          // statistics of the values actually stored, about the pivots
          const f32x2 g01 = bf2_to_f2(o.x), g23 = bf2_to_f2(o.y);
          const f32x2 d01 = g01 - f32x2{c1.x, c1.y}, d23 = g23 - f32x2{c1.z, c1.w};
          sa[i][0] += d01; sa[i][1] += d23;
          sb[i][0] += d01 * d01; sb[i][1] += d23 * d23;
        } else if constexpr (MODE == 2) {
          const f32x2 g01 = bf2_to_f2(o.x), g23 = bf2_to_f2(o.y);
          const f32x2 x01 = bf2_to_f2(ec[NE > 1 ? 1 : 0][i][j].x), x23 = bf2_to_f2(ec[NE > 1 ? 1 : 0][i][j].y);
          const f32x2 h01 = (x01 - f32x2{c0.x, c0.y}) * f32x2{c1.x, c1.y};
          const f32x2 h23 = (x23 - f32x2{c0.z, c0.w}) * f32x2{c1.z, c1.w};
          sa[i][0] += g01; sa[i][1] += g23;
          sb[i][0] += g01 * h01; sb[i][1] += g23 * h23;
        }
      }
    }
    if (STG) {
#pragma unroll
      for (int k = 0; k < TP / 8; ++k) {
        const int P = k * 8 + (lane >> 3), c = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(stg + P * 128 + ((c ^ (P & 7)) << 4));
        *reinterpret_cast<uint4*>(p.Y + (size_t)orow(t * TP + P) * p.N + n0 + c * 8) = v;
      }
    }
  };

  if constexpr (WL) {
    if (t0 < t1) load_chunk(bq[0], t0, 0);
  } else {
#pragma unroll
    for (int d = 0; d < (PF > 1 ? PF - 1 : 1); ++d)
      if (t0 + d < t1) load_b(bb[d], t0 + d);
  }
  if (EP && has_e && t0 < t1) load_e(eo[0], t0);
  if constexpr (PF == 1) {
    for (int t = t0; t < t1; ++t) tile(t, bb[0], bb[0], eo[0], eo[0]);
  } else for (int t = t0; t < t1; t += PF) {
    tile(t, bb[0], bb[PF - 1], eo[0], eo[1]);
    if (t + 1 >= t1) break;
    tile(t + 1, bb[1 % PF], bb[0], eo[1], eo[0]);
    if constexpr (PF == 4) {
      if (t + 2 >= t1) break;
      tile(t + 2, bb[2 % PF], bb[1], eo[0], eo[1]);
      if (t + 3 >= t1) break;
      tile(t + 3, bb[3 % PF], bb[2 % PF], eo[1], eo[0]);
    }
  }
  if constexpr (MODE != 0) {
    const float npx = (float)((t1 - t0) * TP);  // (0 for an empty trailing range: a zero row)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = g1_row_sum(r < 2 ? sa[i][0][r] : sa[i][1][r - 2]);
        const float q = g1_row_sum(r < 2 ? sb[i][0][r] : sb[i][1][r - 2]);
        if (lr == 0) {
          const int c = n0 + i * 16 + lh * 4 + r;
          if constexpr (MODE == 1) {
            store_welford(p.stats, pr, p.N, c, welford_from_shifted(npx, cst[wid][1][c - n0], a, q));
          } else {
            p.stats[((long)pr * 2 + 0) * p.N + c] = a;
            p.stats[((long)pr * 2 + 1) * p.N + c] = q;
          }
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int g_g1s = 1;  // g1s_enable(0): 1x1 convs back on the gathered GEMM (test hook)
void g1s_enable(int on) { g_g1s = on; }

// statistics rows (= pixel ranges) of a streaming 1x1 conv with M output pixels, N output and K
// input channels in `mode`; 0 when the shape does not run on it. The ranges are sized so every
// resident wave slot holds one wave (two per SIMD when the registers allow, else one).
int g1s_rows(int M, int N, int K, int mode) {
  if (!g_g1s || M % 64 || N % 64 || (K != 32 && K != 64 && K != 128 && K != 256 && K != 512)) return 0;
  const int tiles = M / kG1sTile, CS = N / 64;
  const long waves = 256l * 4 * g1s_occ_rt(K, mode);
  int pr = (int)((waves + CS - 1) / CS);
  if (pr > tiles) pr = tiles;
  const int tpr = (tiles + pr - 1) / pr;
  pr = (tiles + tpr - 1) / tpr;
  if (g1s_wl(K, mode)) pr = (pr + 3) / 4 * 4;  // 4 pixel ranges per workgroup (trailing ones may be empty)
  return pr;
}
static int g1s_tpr(int M, int N, int K, int mode) {
  const int tiles = M / kG1sTile, CS = N / 64;
  const long waves = 256l * 4 * g1s_occ_rt(K, mode);
  int pr = (int)((waves + CS - 1) / CS);
  if (pr > tiles) pr = tiles;
  return (tiles + pr - 1) / pr;
}

template <int K, int MODE, int OCC = 2>
static void launch_g1s(const G1sArgs& a, hipStream_t s) {
  const int waves = a.PR * (a.N / 64);
  if (a.gen) {  // gathered stride-phase form: single B buffer (its addressing needs the registers)
    if constexpr (MODE != 1)
      hipLaunchKernelGGL((g1s_kernel<K, MODE, OCC, 1, false, true>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
    DCNN_LAUNCH_CHECK();
    return;
  }
  // B fragments two tiles deep; epilogue operands (residual / BatchNorm y, x) one tile ahead only
  // with DCNN_G1S_PF=3 (more registers: spills on the wider instances)
  // (K >= 128: one B buffer, reloaded after the MFMAs — the two-deep ring spills there)
  if (K >= 128)
    hipLaunchKernelGGL((g1s_kernel<K, MODE, OCC, 1, false>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((g1s_kernel<K, MODE, OCC, 2, false>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
  DCNN_LAUNCH_CHECK();
}

// mode: 0 plain, 1 forward + Welford statistics ([rows][3][N]), 2 data gradient + bnb sums
// ([rows][2][N]); rows must be g1s_rows(M, N, K)
static void g1s_launch(G1sArgs& a, int mode, hipStream_t s) {
  const int K = a.K;
  const int rows = g1s_rows(a.M, a.N, K, mode);
  if (!rows) throw std::runtime_error("g1s: unsupported shape");
  if (mode < 0 || mode > 2 || (mode != 0 && !a.stats)) throw std::runtime_error("g1s: bad mode / statistics slab");
  if (mode == 2 && (!a.bnb.x || !a.bnb.mean || !a.bnb.istd)) throw std::runtime_error("g1s: bnb operands missing");
  if (mode == 1 && a.residual) throw std::runtime_error("g1s: no residual with forward statistics");
  if (mode != 0 && a.relu) throw std::runtime_error("g1s: ReLU only without statistics");
  a.tiles = a.M / kG1sTile;
  a.tpr = g1s_tpr(a.M, a.N, K, mode);
  a.PR = rows;
#define DCNN_G1S(K_)                                          \
  if (K == K_) {                                              \
    if (mode == 0) return launch_g1s<K_, 0>(a, s);            \
    if (mode == 1) return launch_g1s<K_, 1>(a, s);            \
    return launch_g1s<K_, 2>(a, s);                           \
  }
  DCNN_G1S(32)
  DCNN_G1S(64)
  DCNN_G1S(128)
  DCNN_G1S(256)
  DCNN_G1S(512)
#undef DCNN_G1S
  throw std::runtime_error("g1s: no kernel instance");
}

void g1s(const bf16* X, const bf16* Wt, bf16* Y, int M, int N, int K, int H, int W, int OH, int OW, int S,
         const float* bias, const bf16* residual, float* stats, int relu, float* zero_ptr, int zero_n, BnbArgs bnb,
         int mode, hipStream_t s) {
  if (mode == 2 && S != 1) throw std::runtime_error("g1s: bnb fusion needs stride 1 (use g1s_gen)");
  if ((long)M != (long)(M / (OH * OW)) * OH * OW || OH != (H - 1) / S + 1 || OW != (W - 1) / S + 1)
    throw std::runtime_error("g1s: inconsistent geometry");
  G1sArgs a{};
  a.X = X; a.Wt = Wt; a.Y = Y;
  a.M = M; a.N = N; a.K = K; a.H = H; a.W = W; a.OH = OH; a.OW = OW; a.S = S;
  a.bias = bias; a.residual = residual; a.stats = stats; a.relu = relu;
  a.zero_ptr = zero_ptr; a.zero_n = zero_n;
  a.bnb = bnb;
  a.gen = 0; a.ntaps = 1; a.Kc = K; a.ldw = K; a.GH = OH; a.GW = OW;
  g1s_launch(a, mode, s);
}

// gathered form: one stride-phase class of a strided data gradient (see G1sArgs)
int g1s_gen_rows(int M, int N, int Kc, int ntaps, int mode) {
  if (Kc % 32 || ntaps < 0 || ntaps > 4) return 0;
  return g1s_rows(M, N, ntaps == 0 ? 32 : ntaps * Kc, mode);
}

void g1s_gen(const bf16* X, const bf16* Wt, bf16* Y, int NB, int GH, int GW, int N, int Kc, int ldw,
             const std::vector<std::array<int, 3>>& taps, int H, int W, int OHo, int OWo, int OS, int ORY, int ORX,
             const bf16* residual, float* stats, float* zero_ptr, int zero_n, BnbArgs bnb, int mode, hipStream_t s) {
  const int nt = (int)taps.size();
  if (nt > 4 || Kc % 32) throw std::runtime_error("g1s_gen: at most 4 taps of 32-multiple channels");
  if (mode == 1) throw std::runtime_error("g1s_gen: data-gradient modes only (0 / 2)");
  for (int t = 0; t < nt; ++t)
    if (taps[t][2] < 0 || taps[t][2] + Kc > ldw) throw std::runtime_error("g1s_gen: tap weight columns out of the row");
  G1sArgs a{};
  a.X = X; a.Wt = Wt; a.Y = Y;
  a.M = NB * GH * GW; a.N = N; a.K = nt == 0 ? 32 : nt * Kc;
  a.H = H; a.W = W; a.OH = GH; a.OW = GW; a.S = 1;
  a.residual = residual; a.stats = stats; a.zero_ptr = zero_ptr; a.zero_n = zero_n; a.bnb = bnb;
  a.gen = 1; a.ntaps = nt; a.Kc = nt == 0 ? 32 : Kc; a.ldw = ldw;
  a.GH = GH; a.GW = GW; a.OS = OS; a.ORY = ORY; a.ORX = ORX; a.OHo = OHo; a.OWo = OWo;
  for (int t = 0; t < nt; ++t) { a.tap_dy[t] = taps[t][0]; a.tap_dx[t] = taps[t][1]; a.tap_k[t] = taps[t][2]; }
  if (nt == 0) a.ldw = 32;  // (no weight reads happen; keeps wcol in range)
  g1s_launch(a, mode, s);
}

}  // namespace dcnn
