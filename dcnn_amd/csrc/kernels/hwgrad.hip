// Halo-tiled weight gradient for stride-1 convolutions with a 1-pixel reach (3x3 pad 1) on
// CDNA4 MFMA 16x16x32 bf16 — the wgrad counterpart of hconv.hip.
//
//   dW[co][t][ci] = sum_p dY[p][co] * X[p + off_t][ci]
//
// The gathered TN GEMM (gemm2.hip, gemm_t2) streams one (dY, X-gather) pair per tap column
// block, i.e. the input is re-read 9x through L2 (~64 flop/byte). Here a workgroup owns a
// 64(co) x 9(taps) x 64(ci) block of dW and a run of spatial pixel tiles (IMG x TH x TW = 128
// pixels). Per tile it stages the dY tile [128 px][64 co] and the X halo
// [(TH+2)(TW+2) px][64 ci] into LDS once (16-byte direct-to-LDS loads, zero-filled padding,
// a 3-stage ring so two tiles are in flight while one is consumed),
// then all 9 taps read their B fragments from the same halo at a per-tap row offset; the dY
// (A) fragments are read once per 32-pixel k-step and reused by the 9 taps (~240 flop/byte).
// Fragments are pixel-major in LDS and read with ds_read_b64_tr_b16 (transposing LDS reads).
//
// Wave w (of 4) owns the 16 input channels w*16..+15 of every tap: acc[4 co subtiles][9 taps].
// Workgroups of one split (same pixel tiles) are adjacent in the XCD-remapped order, so the
// dY/X tiles they share stay in one XCD's L2. Split-K partials go to an fp32 slab
// [split][Co][9*Cs] (same layout as gemm_t2) reduced by splitk_reduce.
#include <type_traits>

#include "common.h"
#include "api.h"

namespace dcnn {

namespace {
constexpr unsigned kOOBw = 0x80000000u;
constexpr int PT = 128;  // pixels per spatial tile (GEMM K per tile)

__device__ __forceinline__ void glds16w(i32x4 rsrc, char* lds, unsigned voff) { glds16_opaque(rsrc, lds, voff); }

__device__ __forceinline__ int xcd_remap_w(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// 128-byte rows (64 bf16), 16-byte chunk XOR pattern tuned for 4-row transposed reads
__device__ __forceinline__ int wswz(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

// transposed fragment read: this lane gets rows krow..krow+3 (pixels) of column col0 + (lane & 15)
__device__ __forceinline__ bf16x4 tr4(const char* base, int row, int col) {
  const int chn = col >> 3, within = (col & 7) * 2;
  const char* addr = base + row * 128 + ((chn ^ wswz(row)) << 4) + within;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(const_cast<char*>(addr)));
}
}  // namespace

// compile-time tile geometry (TW x TH pixels x IMG images = 128): every per-lane index in the
// prologue folds to shifts / constant multiplies — with one wave per SIMD nothing hides a long
// integer-division prologue
template <int TW, int TH, int IMG>
struct HWGeo {
  static constexpr int HW2 = TW + 2, HPI = (TH + 2) * HW2, HP = IMG * HPI;
  static constexpr int HNI = (HP + 31) / 32;  // halo glds per wave per tile
  static constexpr int HPR = HNI * 32;        // halo rows in LDS
  static constexpr int TPX = TH * TW;
  static constexpr int STAGE = PT * 128 + HPR * 128;
  static constexpr int EPI_TAPS = (2 * STAGE) / (64 * 68 * 4);  // taps staged per epilogue pass
  static_assert(TPX * IMG == PT, "tile must hold 128 pixels");
};

// NS = LDS stages of the (dY, halo) tile ring: NS - 1 tiles are in flight while one is consumed
// (3 stages: 120-156 KB of LDS, still one workgroup per CU as with 2)
template <int TW, int TH, int IMG, int NS>
__global__ void __launch_bounds__(256, 1) hwgrad_kernel(HWArgs p) {
  using G = HWGeo<TW, TH, IMG>;
  constexpr int HNI = G::HNI, HW2 = G::HW2, HPI = G::HPI, HP = G::HP, TPX = G::TPX, STAGE = G::STAGE;
  constexpr int INS = 4 + HNI;  // direct-to-LDS loads per lane per tile (the vmcnt unit)
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int co_tiles = p.Co / 64, ci_chunks = p.Cs / 64;
  const int per_split = co_tiles * ci_chunks;
  const int lt = xcd_remap_w(blockIdx.x, gridDim.x);
  const int split = lt / per_split, rem = lt - split * per_split;
  const int pair = blockIdx.y, nsplits = gridDim.x / per_split;
  const int yoff = p.pair_yoff[pair], xoff = p.pair_xoff[pair];
  const int co0 = (rem / ci_chunks) * 64, c0 = (rem % ci_chunks) * 64;

  const int tx_tiles = p.W / TW, ty_tiles = p.H / TH, tpi = tx_tiles * ty_tiles;
  const int total_tiles = (p.NB / IMG) * tpi;
  const int tbeg = split * p.tiles_per_split;
  const int tend = min(total_tiles, tbeg + p.tiles_per_split);

  const i32x4 rsY = raw_rsrc(p.dY, p.dy_bytes);
  const i32x4 rsX = raw_rsrc(p.X, p.x_bytes);

  // ---- dY loader: 4 glds per lane, rows (pixels) fixed relative to the tile origin ----
  const int slot = lane & 7;
  unsigned y_rel[4], y_col[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int im = row / TPX, r2 = row - im * TPX;
    y_rel[i] = (unsigned)((im * p.H + r2 / TW) * p.W + r2 % TW);
    y_col[i] = (unsigned)((yoff + co0 + ((slot ^ wswz(row)) * 8)) * 2);
  }
  // ---- halo loader: row (im, hy, hx) of each lane fixed; only the validity test and a
  //      uniform base move with the tile (6 VALU per 16-byte load) ----
  int h_rel[HNI], h_hy[HNI], h_hx[HNI];
#pragma unroll
  for (int j = 0; j < HNI; ++j) {
    const int row = (wid * HNI + j) * 8 + (lane >> 3);
    const int im = row / HPI, r2 = row - im * HPI;
    const int hy = r2 / HW2 - 1, hx = r2 % HW2 - 1;
    const bool real = row < HP;
    h_hy[j] = real ? hy : -(1 << 20);  // padding rows of the buffer: never valid
    h_hx[j] = hx;
    h_rel[j] = ((im * p.H + hy) * p.W + hx) * p.ldx * 2 + (xoff + c0 + ((slot ^ wswz(row)) * 8)) * 2;
  }
  auto load_tile = [&](int buf, int tile) {
    char* Ys = smem + buf * STAGE;
    char* Hs = Ys + PT * 128;
    const int ig = tile / tpi, tr = tile - ig * tpi;
    const int y0 = (tr / tx_tiles) * TH, x0 = (tr % tx_tiles) * TW;
    const int g0 = (ig * IMG * p.H + y0) * p.W + x0;  // tile origin pixel
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16w(rsY, Ys + (wid * 4 + i) * 1024, (unsigned)(g0 + y_rel[i]) * (unsigned)(p.ldy * 2) + y_col[i]);
    const int gx = g0 * p.ldx * 2;
#pragma unroll
    for (int j = 0; j < HNI; ++j) {
      const bool ok = (unsigned)(y0 + h_hy[j]) < (unsigned)p.H && (unsigned)(x0 + h_hx[j]) < (unsigned)p.W;
      glds16w(rsX, Hs + (wid * HNI + j) * 1024, ok ? (unsigned)(gx + h_rel[j]) : kOOBw);
    }
  };

  // ---- per-lane halo row of tap (0,0) for each of the 8 (k-step, half) pixel quads ----
  int hrow[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int px = (s >> 1) * 32 + 8 * (lane >> 4) + (s & 1) * 4 + ((lane & 15) >> 2);
    const int im = px / TPX, r2 = px - im * TPX;
    hrow[s] = im * HPI + (r2 / TW + 1) * HW2 + (r2 % TW + 1);
  }
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) toff[t] = p.tap_dy[t] * HW2 + p.tap_dx[t];

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int bcol = wid * 16 + 4 * (lane & 3);  // B column (input channel) this lane reads
  const bool do_bias = p.bias_slab != nullptr && c0 == 0;
  float bias_acc = 0.f;
  const int nt = tend - tbeg;
  // tile it lives in stage it % NS; tile it + NS - 1 is issued at the top of iteration it into
  // the stage iteration it - 1 consumed (the barrier closing it - 1 retired every read of it)
  if (nt > 0) load_tile(0, tbeg);
  if (NS == 3 && nt > 1) load_tile(1, tbeg + 1);
  if (NS == 3 && nt > 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INS) : "memory");  // tile 0 landed, tile 1 may fly
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int it = 0; it < nt; ++it) {
    if (it + NS - 1 < nt) load_tile(cur == 0 ? NS - 1 : cur - 1, tbeg + it + NS - 1);
    const char* Ys = smem + cur * STAGE;
    const char* Hs = Ys + PT * 128;
    // software pipeline over the 4 k-steps: the fragments of step kk+1 are read while the 36
    // MFMAs of step kk run (one wave per SIMD: nothing else hides the LDS latency)
    bf16x8 a[2][4], b[2][9];
    auto read_step = [&](int kk, bf16x8* av, bf16x8* bv) {
      const int krow = kk * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * (lane & 3);
        const bf16x4 lo = tr4(Ys, krow, col), hi = tr4(Ys, krow + 4, col);
        av[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const bf16x4 lo = tr4(Hs, hrow[kk * 2] + toff[t], bcol), hi = tr4(Hs, hrow[kk * 2 + 1] + toff[t], bcol);
        bv[t] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    read_step(0, a[0], b[0]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int c = kk & 1;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): step kk's fragments have landed
      if (kk + 1 < 4) read_step(kk + 1, a[c ^ 1], b[c ^ 1]);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][i], b[c][t], acc[i][t], 0, 0, 0);
      if (kk + 1 < 4) {
        // interleave: the 26 fragment reads of step kk+1 (and their address VALU) issue in the
        // shadow of step kk's MFMAs instead of in front of them (in-order issue, 1 wave/SIMD)
#pragma unroll
        for (int g = 0; g < 26; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
      }
    }
    if (do_bias) {  // bias gradient: column sums of the staged dY tile (first ci chunk only)
      const int col = tid & 63, chn = col >> 3, w = (col & 7) * 2;
      for (int r = tid >> 6; r < PT; r += 4)
        bias_acc += (float)*reinterpret_cast<const bf16*>(Ys + r * 128 + ((chn ^ wswz(r)) << 4) + w);
    }
    // tile it + 1 must have landed (this lane's loads, then the barrier for everyone's); with 3
    // stages the loads of tile it + 2, issued after it, may stay in flight
    if (NS == 3 && it + 2 < nt)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    cur = cur == NS - 1 ? 0 : cur + 1;
  }

  // ---- slab[split][co][t*Cs + ci]: taps staged through LDS (pitch 68 floats) so every lane
  //      stores 16 contiguous bytes and each 16-lane group a whole 256-byte row segment ----
  const long Ng = 9l * p.Cs;
  const long slab_idx = (long)pair * nsplits + split;
  float* out = p.slab + slab_idx * p.Co * Ng;
  float* stg = reinterpret_cast<float*>(smem);
  constexpr int ET = G::EPI_TAPS;
#pragma unroll
  for (int t0 = 0; t0 < 9; t0 += ET) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < ET; ++u) {
      if (t0 + u < 9) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(u * 64 + i * 16 + (lane >> 4) * 4 + r) * 68 + wid * 16 + (lane & 15)] = acc[i][t0 + u][r];
      }
    }
    __syncthreads();
    const int nrows = (9 - t0 < ET ? 9 - t0 : ET) * 64;
    for (int q = tid; q < nrows * 16; q += 256) {
      const int row = q >> 4, c4 = (q & 15) * 4;
      const int u = row >> 6, co = co0 + (row & 63);
      const float4 v = *reinterpret_cast<const float4*>(stg + row * 68 + c4);
      *reinterpret_cast<float4*>(out + (long)co * Ng + (t0 + u) * p.Cs + c0 + c4) = v;
    }
  }
  if (do_bias) {
    __syncthreads();
    stg[tid] = bias_acc;
    __syncthreads();
    if (tid < 64)
      p.bias_slab[slab_idx * p.Co + co0 + tid] =
          p.pair_bias[pair] ? stg[tid] + stg[tid + 64] + stg[tid + 128] + stg[tid + 192] : 0.f;
  }
}

// ---------------------------------------------------------------------------------------------
// Variant with tap-shift-invariant LDS addressing (hwgrad2): the halo's pixel rows are padded to
// HW2P = round_up(TW + 2, 8) LDS rows and the 16-byte chunk swizzle depends only on row bits 1-2,
// so a tap's dy shift (dy * HW2P rows) leaves the swizzle unchanged and becomes an immediate
// ds_read offset; the three dx shifts get a base address each. Per 128-pixel tile the 104
// fragment reads then need 32 base registers and no per-read address arithmetic (the first
// kernel computes ~180 address VALU per tile and keeps 72 hoisted addresses live, 479 registers).
// The pixel -> MFMA-k mapping puts pixels p..p+7 of an image row in one 32-lane read group
// (rows r..r+7: same-parity rows r, r+2, r+4, r+6 differ in bits 1-2 -> conflict-free).
// Standard 3x3 / pad-1 taps only (t = ky * 3 + kx, dy = ky - 1, dx = kx - 1).
// ---------------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ int wswz2(int row) { return ((row >> 1) & 3) << 1; }
}  // namespace

template <int TW, int TH, int IMG>
struct HWGeo2 {
  static constexpr int HW2P = ((TW + 2 + 7) / 8) * 8, HPIP = (TH + 2) * HW2P, HPP = IMG * HPIP;
  static constexpr int HNI = (HPP + 31) / 32;
  static constexpr int HPR = HNI * 32;
  static constexpr int TPX = TH * TW;
  static constexpr int STAGE = PT * 128 + HPR * 128;
  static constexpr int EPI_TAPS = (2 * STAGE) / (64 * 68 * 4);
  static_assert(TPX * IMG == PT, "tile must hold 128 pixels");
  // (TW = 4: a 32-lane read group spans two image rows, 8 halo rows apart: 2-way LDS conflicts
  // on those reads, accepted — the addressing savings are the same)
};

template <int K, int N, class F>
__device__ __forceinline__ void h3w_static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    h3w_static_for<K + 1, N>(f);
  }
}

__device__ __forceinline__ bf16x4 tr4_at(const char* addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(const_cast<char*>(addr)));
}

// TSP = 2: 8 waves, two per SIMD — wave w + 4 shares wave w's 16 input channels and takes taps
// 5..8 while wave w takes 0..4 (20 / 16 accumulator tiles instead of 36), so a SIMD always has a
// second wave to issue while one waits on LDS or the tile barrier (the 4-wave kernel runs one
// wave per SIMD: every wait is exposed). TSP = 3: 12 waves, taps in thirds. The first four waves
// issue the tile loads. Measured (batch 256): TSP 2 wgrad l1..l4 42.5/35.3/37.4/40.0 ->
// 40.8/33.7/35.5/38.1 us, whole step 78.3k -> 80.0k img/s.
// F32: exact fp32 operands (hwgrad_f32). As in hconv3's fp32 instances, an fp32 row of C channels
// is a bf16 row of 2C byte for byte, so the launcher passes 2 Co / 2 Cs / 2 ldy / 2 ldx and the
// staging (DMA pieces, swizzle, halo rows) is the bf16 one; a workgroup then owns 32 (co) x 9 x
// 32 (ci) fp32 outputs. The fragments are single fp32 values (ds_read_b32, no transposing read) for
// v_mfma_f32_16x16x4_f32: wave w takes co half w >> 1 and ci half w & 1 (one 16x16 tile per tap),
// MFMA k0 (of 4 per 16-pixel block) takes pixels k0 + 4 lh — 4 rows apart, so the two pixels of a
// 32-lane read group sit in chunk-swizzle classes 4 apart and hit disjoint banks.
// C32: Cs = 32 (one 64-channel chunk, the upper half read as zeros and not stored); its own
// instances, so the compare stays out of the others (ResNet-50 b32 measured -0.3% with it inline)
template <int TW, int TH, int IMG, int NS, int TSP = 1, bool F32 = false, bool C32 = false>
__global__ void __launch_bounds__(256 * TSP, 1) hwgrad2_kernel(HWArgs p) {
  prefetch_kernargs<sizeof(HWArgs)>();
  using G = HWGeo2<TW, TH, IMG>;
  constexpr int HNI = G::HNI, HW2P = G::HW2P, HPIP = G::HPIP, HPP = G::HPP, TPX = G::TPX, STAGE = G::STAGE;
  constexpr int INS = 4 + HNI;
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = (tid >> 6) & 3, th = tid >> 8;
  constexpr int NT = 256 * TSP;
  // (Cs = 32: one 64-channel chunk whose upper half reads zeros and is not stored — ResNet-18's
  // first residual conv, 32 input channels)
  const int co_tiles = p.Co / 64, ci_chunks = (p.Cs + 63) / 64;
  const int per_split = co_tiles * ci_chunks;
  const int lt = xcd_remap_w(blockIdx.x, gridDim.x);
  const int split = lt / per_split, rem = lt - split * per_split;
  const int pair = blockIdx.y, nsplits = gridDim.x / per_split;
  const int yoff = p.pair_yoff[pair], xoff = p.pair_xoff[pair];
  const int co0 = (rem / ci_chunks) * 64, c0 = (rem % ci_chunks) * 64;

  const int tx_tiles = p.W / TW, ty_tiles = p.H / TH, tpi = tx_tiles * ty_tiles;
  const int total_tiles = (p.NB / IMG) * tpi;
  const int tbeg = split * p.tiles_per_split;
  const int tend = min(total_tiles, tbeg + p.tiles_per_split);
  const i32x4 rsY = raw_rsrc(p.dY, p.dy_bytes);
  const i32x4 rsX = raw_rsrc(p.X, p.x_bytes);

  // ---- dY loader (tile rows = pixels, 128 B each) ----
  const int slot = lane & 7;
  unsigned y_rel[4], y_col[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int im = row / TPX, r2 = row - im * TPX;
    y_rel[i] = (unsigned)((im * p.H + r2 / TW) * p.W + r2 % TW);
    y_col[i] = (unsigned)((yoff + co0 + ((slot ^ wswz2(row)) * 8)) * 2);
  }
  // ---- halo loader: padded rows (hx >= TW + 1) are never valid ----
  int h_rel[HNI], h_hy[HNI], h_hx[HNI];
#pragma unroll
  for (int j = 0; j < HNI; ++j) {
    const int row = (wid * HNI + j) * 8 + (lane >> 3);
    const int im = row / HPIP, r2 = row - im * HPIP;
    const int hy = r2 / HW2P - 1, hx = r2 % HW2P - 1;
    const bool real = row < HPP && hx <= TW && (!C32 || c0 + ((slot ^ wswz2(row)) * 8) < p.Cs);
    h_hy[j] = real ? hy : -(1 << 20);
    h_hx[j] = hx;
    h_rel[j] = ((im * p.H + hy) * p.W + hx) * p.ldx * 2 + (xoff + c0 + ((slot ^ wswz2(row)) * 8)) * 2;
  }
  auto load_tile = [&](int buf, int tile) {
    if (TSP > 1 && th != 0) return;
    char* Ys = smem + buf * STAGE;
    char* Hs = Ys + PT * 128;
    const int ig = tile / tpi, tr = tile - ig * tpi;
    const int y0 = (tr / tx_tiles) * TH, x0 = (tr % tx_tiles) * TW;
    const int g0 = (ig * IMG * p.H + y0) * p.W + x0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16w(rsY, Ys + (wid * 4 + i) * 1024, (unsigned)(g0 + y_rel[i]) * (unsigned)(p.ldy * 2) + y_col[i]);
    const int gx = g0 * p.ldx * 2;
#pragma unroll
    for (int j = 0; j < HNI; ++j) {
      const bool ok = (unsigned)(y0 + h_hy[j]) < (unsigned)p.H && (unsigned)(x0 + h_hx[j]) < (unsigned)p.W;
      glds16w(rsX, Hs + (wid * HNI + j) * 1024, ok ? (unsigned)(gx + h_rel[j]) : kOOBw);
    }
  };

  // the first tile(s) go out before the fragment-address arithmetic below (both run variants start
  // with them; only ALU work sits between here and their counted waits)
  const int nt = tend - tbeg;
  if (nt > 0) load_tile(0, tbeg);
  if (NS == 3 && nt > 1) load_tile(1, tbeg + 1);

  // ---- fragment base addresses (stage-relative bytes) ----
  // pixel of (k-step kk, half h) for this lane: kk*32 + h*16 + 4*(lane>>4) + ((lane&15)>>2)
  const int lpx = 4 * (lane >> 4) + ((lane & 15) >> 2);
  // A (dY tile): row = kk*32 + h*16 + lpx, column i*16 + 4*(lane&3); kk and h shift the row by
  // multiples of 8 (swizzle unchanged) -> immediate offsets kk*4096 + h*2048
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + 4 * (lane & 3);
    abase[i] = lpx * 128 + (((col >> 3) ^ wswz2(lpx)) << 4) + (col & 7) * 2;
  }
  // B (halo): row of pixel px, tap (dy, dx) = hrow(px) + dy*HW2P + dx; base per (kk, h, dx) at
  // dy = -1, dy = 0 / +1 as immediate offsets HW2P*128 / 2*HW2P*128
  const int bcol = wid * 16 + 4 * (lane & 3);
  int bbase[8][3];
#pragma unroll
  for (int sidx = 0; sidx < 8; ++sidx) {
    const int px = (sidx >> 1) * 32 + (sidx & 1) * 16 + lpx;
    const int im = px / TPX, r2 = px - im * TPX;
    const int hr = im * HPIP + (r2 / TW + 1) * HW2P + r2 % TW + 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int row = hr + (d - 1) - HW2P;  // dx = d - 1, dy = -1
      bbase[sidx][d] = PT * 128 + row * 128 + (((bcol >> 3) ^ wswz2(row)) << 4) + (bcol & 7) * 2;
    }
  }

  // F32 fragment bases: pixel (block b, MFMA k0, lane group lh) = 16 b + k0 + 4 lh; the block's
  // rows are a compile-time offset (a multiple of 8 LDS rows: the swizzle is unchanged)
  int fa[4], fb[4][3];
  const int fco = 16 * (wid >> 1) + (lane & 15), fci = 16 * (wid & 1) + (lane & 15);  // fp32 columns
  if constexpr (F32) {
#pragma unroll
    for (int k0 = 0; k0 < 4; ++k0) {
      const int px = k0 + 4 * (lane >> 4);  // pixel within the 16-pixel block
      fa[k0] = px * 128 + (((fco >> 2) ^ wswz2(px)) << 4) + (fco & 3) * 4;
      // halo row of the block-0 pixel px at tap (dy, dx) = (-1, d - 1)
      int hr0;
      if constexpr (TW == 16) hr0 = HW2P + px + 1;                             // row 0 of the tile
      else if constexpr (TW == 8) hr0 = ((px >> 3) + 1) * HW2P + (px & 7) + 1;  // rows 0-1
      else hr0 = ((px >> 2) + 1) * HW2P + (px & 3) + 1;                         // TW 4: image 0, rows 0-3
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int row = hr0 + (d - 1) - HW2P;
        fb[k0][d] = PT * 128 + row * 128 + (((fci >> 2) ^ wswz2(row)) << 4) + (fci & 3) * 4;
      }
    }
  }
  // halo-row offset of 16-pixel block b relative to block 0 (compile time)
  auto blk_rows = [](int b) constexpr {
    if (TW == 16) return b * HW2P;                                    // one image row per block
    if (TW == 8) return (b / 4) * HPIP + (b % 4) * 2 * HW2P;         // 2 rows per block, 4 per image
    return b * HPIP;                                                   // TW 4: one image per block
  };

  // the tile loop and epilogue for taps TB .. TB + NTW - 1 (compile-time: register arrays indexed
  // by tap stay static)
  auto run_f32 = [&](auto tb_c, auto ntw_c) {
    constexpr int TB = decltype(tb_c)::value, NTW = decltype(ntw_c)::value;
    f32x4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = p.bias_slab != nullptr && c0 == 0 && th == 0;
    float bias_acc = 0.f;
    if (NS == 3 && nt > 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < nt; ++it) {
      if (it + NS - 1 < nt) load_tile(cur == 0 ? NS - 1 : cur - 1, tbeg + it + NS - 1);
      const char* S0 = smem + cur * STAGE;
      auto lds_f = [&](int off) { return *reinterpret_cast<const float*>(S0 + off); };
      float a[2], b[2][NTW];
      auto rd = [&](auto blk_c, int k0, int c) {
        constexpr int B = decltype(blk_c)::value;
        a[c] = lds_f(fa[k0] + B * 16 * 128);
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const int tt = TB + t, dy = tt / 3, dx = tt % 3;
          b[c][t] = lds_f(fb[k0][dx] + (blk_rows(B) + dy * HW2P) * 128);
        }
      };
      h3w_static_for<0, 8>([&](auto blk_c) {
        constexpr int B = decltype(blk_c)::value;
        rd(blk_c, 0, 0);
#pragma unroll
        for (int k0 = 0; k0 < 4; ++k0) {
          const int c = k0 & 1;
          if (k0 + 1 < 4) rd(blk_c, k0 + 1, c ^ 1);
#pragma unroll
          for (int t = 0; t < NTW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b[c][t], acc[t], 0, 0, 0);
        }
        (void)B;
      });
      if (do_bias) {  // dY column sums: thread -> fp32 column tid & 31, rows (tid >> 5) + 8 r
        const int col = tid & 31;
        for (int r = tid >> 5; r < PT; r += 8)
          bias_acc += *reinterpret_cast<const float*>(S0 + r * 128 + (((col >> 2) ^ wswz2(r)) << 4) + (col & 3) * 4);
      }
      if (NS == 3 && it + 2 < nt)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
    // ---- slab[split][co][t * Cs + ci] in fp32 units (Co / Cs of the launcher are doubled)
    const int Cs = p.Cs / 2, Co = p.Co / 2, cof = co0 / 2, cif = c0 / 2;
    const long Ng = 9l * Cs;
    const long slab_idx = (long)pair * nsplits + split;
    float* out = p.slab + slab_idx * Co * Ng;
    float* stg = reinterpret_cast<float*>(smem);
    constexpr int ET = G::EPI_TAPS;
#pragma unroll
    for (int t0 = 0; t0 < 9; t0 += ET) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < ET; ++u) {
        const int tl = t0 + u - TB;
        if (t0 + u < 9 && tl >= 0 && tl < NTW) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(u * 32 + 16 * (wid >> 1) + (lane >> 4) * 4 + r) * 36 + 16 * (wid & 1) + (lane & 15)] = acc[tl][r];
        }
      }
      __syncthreads();
      const int nrows = (9 - t0 < ET ? 9 - t0 : ET) * 32;
      for (int q = tid; q < nrows * 8; q += NT) {
        const int row = q >> 3, c4 = (q & 7) * 4;
        const int u = row >> 5, co = cof + (row & 31);
        const float4 v = *reinterpret_cast<const float4*>(stg + row * 36 + c4);
        *reinterpret_cast<float4*>(out + (long)co * Ng + (t0 + u) * Cs + cif + c4) = v;
      }
    }
    if (p.bias_slab != nullptr && c0 == 0) {
      __syncthreads();
      if (tid < 256) stg[tid] = bias_acc;
      __syncthreads();
      if (tid < 32) {
        float sum = 0.f;
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) sum += stg[gi * 32 + tid];
        p.bias_slab[slab_idx * Co + cof + tid] = p.pair_bias[pair] ? sum : 0.f;
      }
    }
  };
  auto run = [&](auto tb_c, auto ntw_c) {
    constexpr int TB = decltype(tb_c)::value, NTW = decltype(ntw_c)::value;
    f32x4 acc[4][NTW];
  #pragma unroll
    for (int i = 0; i < 4; ++i)
  #pragma unroll
      for (int t = 0; t < NTW; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const bool do_bias = p.bias_slab != nullptr && c0 == 0 && th == 0;
    float bias_acc = 0.f;
    if (NS == 3 && nt > 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    for (int it = 0; it < nt; ++it) {
      if (it + NS - 1 < nt) load_tile(cur == 0 ? NS - 1 : cur - 1, tbeg + it + NS - 1);
      const char* S0 = smem + cur * STAGE;
      // A double-buffered; each tap's B fragment re-read in place right after the step's 4 MFMAs
      // that consume it (9 live B fragments instead of 18: the multi-image geometries otherwise
      // spill through AGPRs)
      bf16x8 a[2][4], b[NTW];
      auto read_a = [&](int kk, bf16x8* av) {
  #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const char* q = S0 + abase[i] + kk * 4096;
          const bf16x4 lo = tr4_at(q), hi = tr4_at(q + 2048);
          av[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      };
      auto read_b = [&](int kk, int t) {
        const int dy = t / 3, dx = t % 3;
        const bf16x4 lo = tr4_at(S0 + bbase[kk * 2][dx] + dy * HW2P * 128);
        const bf16x4 hi = tr4_at(S0 + bbase[kk * 2 + 1][dx] + dy * HW2P * 128);
        return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      read_a(0, a[0]);
  #pragma unroll
      for (int t = 0; t < NTW; ++t) b[t] = read_b(0, TB + t);
  #pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int c = kk & 1;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        if (kk + 1 < 4) read_a(kk + 1, a[c ^ 1]);
  #pragma unroll
        for (int t = 0; t < NTW; ++t) {
  #pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][i], b[t], acc[i][t], 0, 0, 0);
          if (kk + 1 < 4) b[t] = read_b(kk + 1, TB + t);
        }
      }
      if (do_bias) {
        const int col = tid & 63, chn = col >> 3, w = (col & 7) * 2;
        for (int r = wid; r < PT; r += 4)
          bias_acc += (float)*reinterpret_cast<const bf16*>(S0 + r * 128 + ((chn ^ wswz2(r)) << 4) + w);
      }
      if (NS == 3 && it + 2 < nt)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      cur = cur == NS - 1 ? 0 : cur + 1;
    }

    // ---- slab[split][co][t*Cs + ci] (as hwgrad_kernel) ----
    const long Ng = 9l * p.Cs;
    const long slab_idx = (long)pair * nsplits + split;
    float* out = p.slab + slab_idx * p.Co * Ng;
    float* stg = reinterpret_cast<float*>(smem);
    constexpr int ET = G::EPI_TAPS;
  #pragma unroll
    for (int t0 = 0; t0 < 9; t0 += ET) {
      __syncthreads();
  #pragma unroll
      for (int u = 0; u < ET; ++u) {
        const int tl = t0 + u - TB;  // this wave's accumulator slot of tap t0 + u
        if (t0 + u < 9 && tl >= 0 && tl < NTW) {
  #pragma unroll
          for (int i = 0; i < 4; ++i)
  #pragma unroll
            for (int r = 0; r < 4; ++r)
              stg[(u * 64 + i * 16 + (lane >> 4) * 4 + r) * 68 + wid * 16 + (lane & 15)] = acc[i][tl][r];
        }
      }
      __syncthreads();
      const int nrows = (9 - t0 < ET ? 9 - t0 : ET) * 64;
      for (int q = tid; q < nrows * 16; q += NT) {
        const int row = q >> 4, c4 = (q & 15) * 4;
        const int u = row >> 6, co = co0 + (row & 63);
        const float4 v = *reinterpret_cast<const float4*>(stg + row * 68 + c4);
        if (!C32 || c0 + c4 < p.Cs) *reinterpret_cast<float4*>(out + (long)co * Ng + (t0 + u) * p.Cs + c0 + c4) = v;
      }
    }
    if (p.bias_slab != nullptr && c0 == 0) {  // (every wave passes the same barriers)
      __syncthreads();
      if (tid < 256) stg[tid] = bias_acc;
      __syncthreads();
      if (tid < 64)
        p.bias_slab[slab_idx * p.Co + co0 + tid] =
            p.pair_bias[pair] ? stg[tid] + stg[tid + 64] + stg[tid + 128] + stg[tid + 192] : 0.f;
    }

  };
  if constexpr (F32) {
    static_assert(TSP == 2, "fp32: 8 waves");
    if (th == 0) run_f32(std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{});
    else run_f32(std::integral_constant<int, 5>{}, std::integral_constant<int, 4>{});
  } else if constexpr (TSP == 1) {
    run(std::integral_constant<int, 0>{}, std::integral_constant<int, 9>{});
  } else if constexpr (TSP == 2) {
    if (th == 0) run(std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{});
    else run(std::integral_constant<int, 5>{}, std::integral_constant<int, 4>{});
  } else {
    if (th == 0) run(std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
    else if (th == 1) run(std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{});
    else run(std::integral_constant<int, 6>{}, std::integral_constant<int, 3>{});
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// supported tile geometries (TW, TH, IMG): W multiple of 16 and H of 8; 8x8; 4x4 maps
static bool hw_geometry(int H, int W, int* TH, int* TW, int* IMG) {
  if (W % 16 == 0 && H % 8 == 0) { *TW = 16; *TH = 8; *IMG = 1; return true; }
  if (W == 8 && H == 8) { *TW = 8; *TH = 8; *IMG = 2; return true; }
  if (W == 4 && H == 4) { *TW = 4; *TH = 4; *IMG = 8; return true; }
  return false;
}

static int g_hwgrad_version = 2;  // (hwgrad_set_version below)

bool hwgrad_supported(int NB, int H, int W, int Cs, int Co, int ntaps) {
  int th, tw, img;
  // 3x3 (all 9 taps unrolled); Cs = 32 on the tap-shift-invariant kernel only (a half-empty
  // 64-channel chunk: ResNet-18 layer 1's first conv, 52.8 us on the gathered GEMM)
  if ((Cs % 64 && !(Cs == 32 && g_hwgrad_version == 2)) || Co % 64 || ntaps != 9) return false;
  if (!hw_geometry(H, W, &th, &tw, &img) || NB % img) return false;
  // 32-bit buffer offsets
  return (long)NB * H * W * (Cs > Co ? Cs : Co) * 2 < (1l << 31);
}

static int kHwTargetBlocks = 256;  // split-K target: one workgroup per CU
void hwgrad_set_split_target(int t) { kHwTargetBlocks = t < 1 ? 1 : t; }

// number of split-K partial slabs (the caller sizes the slab [splits][Co][ntaps*Cs])
int hwgrad_splits(int NB, int H, int W, int Cs, int Co) {
  int th, tw, img;
  if (!hw_geometry(H, W, &th, &tw, &img)) return 1;
  const int total = (NB / img) * (H / th) * (W / tw);
  const int per_split = (Co / 64) * ((Cs + 63) / 64);
  int want = (kHwTargetBlocks + per_split - 1) / per_split;
  if (want < 1) want = 1;
  if (want > total) want = total;
  // at least 2 tiles per split: a one-tile block writes ~4.6x the bytes it reads as fp32
  // partials (64x576 per 128 pixels). ResNet-50 batch 32 (one-tile splits on its 32x32 maps):
  // 7.76k -> 7.90k img/s (profiles/wgrad_splits_r3.md)
  constexpr int min_tps = 2;
  if (min_tps > 1 && want > total / min_tps) want = total / min_tps > 1 ? total / min_tps : 1;
  const int tps = (total + want - 1) / want;
  return (total + tps - 1) / tps;
}

// kernel generation: 2 = tap-shift-invariant addressing where it applies (8 waves, taps split
// 0-4 / 5-8 over two waves per SIMD), 1 = first kernel only (test hook)
void hwgrad_set_version(int v) { g_hwgrad_version = v; }

void hwgrad(HWArgs a, int splits, hipStream_t s) {
  if (!hwgrad_supported(a.NB, a.H, a.W, a.Cs, a.Co, a.ntaps)) throw std::runtime_error("hwgrad: unsupported shape");
  for (int t = 0; t < a.ntaps; ++t)
    if (a.tap_dy[t] < -1 || a.tap_dy[t] > 1 || a.tap_dx[t] < -1 || a.tap_dx[t] > 1)
      throw std::runtime_error("hwgrad: taps must reach at most 1 pixel");
  if (splits != hwgrad_splits(a.NB, a.H, a.W, a.Cs, a.Co)) throw std::runtime_error("hwgrad: split count mismatch");
  if (a.npairs == 0) {  // plain wgrad
    a.npairs = 1; a.ldy = a.Co; a.ldx = a.Cs;
    a.pair_yoff[0] = a.pair_xoff[0] = 0; a.pair_bias[0] = 1;
  }
  if (a.npairs < 1 || a.npairs > 3 || a.ldy % 8 || a.ldx % 8) throw std::runtime_error("hwgrad: bad operand pairs");
  for (int q = 0; q < a.npairs; ++q)
    if (a.pair_yoff[q] < 0 || a.pair_yoff[q] + a.Co > a.ldy || a.pair_xoff[q] < 0 || a.pair_xoff[q] + a.Cs > a.ldx ||
        a.pair_yoff[q] % 8 || a.pair_xoff[q] % 8)
      throw std::runtime_error("hwgrad: pair channel window outside the rows");
  if ((long)a.NB * a.H * a.W * (a.ldx > a.ldy ? a.ldx : a.ldy) * 2 >= (1l << 31))
    throw std::runtime_error("hwgrad: operands exceed 32-bit buffer offsets");
  hw_geometry(a.H, a.W, &a.TH, &a.TW, &a.IMG);
  const int total = (a.NB / a.IMG) * (a.H / a.TH) * (a.W / a.TW);
  a.tiles_per_split = (total + splits - 1) / splits;
  const int grid = splits * (a.Co / 64) * ((a.Cs + 63) / 64);
  constexpr int stages = 3;
  // tap-shift-invariant variant (hwgrad2_kernel) for the standard 3x3 / pad-1 taps on 16- and
  // 8-wide maps (hwgrad_set_version(1) keeps the first kernel)
  const int ver = g_hwgrad_version;
  bool std_taps = a.ntaps == 9;
  for (int t = 0; t < a.ntaps && std_taps; ++t) std_taps = a.tap_dy[t] == t / 3 - 1 && a.tap_dx[t] == t % 3 - 1;
  const bool c32 = a.Cs % 64 != 0;
  if (c32 && !(ver == 2 && std_taps)) throw std::runtime_error("hwgrad: Cs = 32 needs the standard 3x3 taps");
  if (ver == 2 && std_taps) {
#define DCNN_HW2(TW_, TH_, IMG_, NS_)                                                                   \
    if (a.TW == TW_ && a.TH == TH_ && a.IMG == IMG_) {                                                  \
      auto k = c32 ? hwgrad2_kernel<TW_, TH_, IMG_, NS_, 2, false, true> : hwgrad2_kernel<TW_, TH_, IMG_, NS_, 2>; \
      const int lds = NS_ * HWGeo2<TW_, TH_, IMG_>::STAGE;                                              \
      DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
      hipLaunchKernelGGL(k, dim3(grid, a.npairs), dim3(512), lds, s, a);                                \
      DCNN_LAUNCH_CHECK();                                                                              \
      return;                                                                                           \
    }
    DCNN_HW2(16, 8, 1, 3)  // 3 x 48 KB
    DCNN_HW2(8, 8, 2, 2)   // 2 x 56 KB (three stages would need 168 KB)
    if (g_hwgrad_version == 2 && a.TW == 4 && a.TH == 4 && a.IMG == 8) {
      auto k = c32 ? hwgrad2_kernel<4, 4, 8, 2, 2, false, true> : hwgrad2_kernel<4, 4, 8, 2, 2>;  // 2 x 64 KB
      const int lds = 2 * HWGeo2<4, 4, 8>::STAGE;
      DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
      hipLaunchKernelGGL(k, dim3(grid, a.npairs), dim3(512), lds, s, a);
      DCNN_LAUNCH_CHECK();
      return;
    }
#undef DCNN_HW2
  }
#define DCNN_HW(TW_, TH_, IMG_, NS_)                                                                    \
  if (a.TW == TW_ && a.TH == TH_ && a.IMG == IMG_ && stages == NS_) {                                   \
    auto k = hwgrad_kernel<TW_, TH_, IMG_, NS_>;                                                        \
    const int lds = NS_ * HWGeo<TW_, TH_, IMG_>::STAGE;                                                 \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(grid, a.npairs), dim3(256), lds, s, a);                                  \
    DCNN_LAUNCH_CHECK();                                                                                \
    return;                                                                                             \
  }
  DCNN_HW(16, 8, 1, 3)
  DCNN_HW(8, 8, 2, 3)
  DCNN_HW(4, 4, 8, 3)
  DCNN_HW(16, 8, 1, 2)
  DCNN_HW(8, 8, 2, 2)
  DCNN_HW(4, 4, 8, 2)
#undef DCNN_HW
  throw std::runtime_error("hwgrad: no kernel for this geometry");
}

bool hwgrad_f32_supported(int NB, int H, int W, int Cs, int Co) {
  int th, tw, img;
  if (Cs % 32 || Co % 32) return false;
  if (!hw_geometry(H, W, &th, &tw, &img) || NB % img) return false;
  return (long)NB * H * W * (Cs > Co ? Cs : Co) * 4 < (1l << 31);
}

int hwgrad_f32_splits(int NB, int H, int W, int Cs, int Co) { return hwgrad_splits(NB, H, W, 2 * Cs, 2 * Co); }

// exact fp32 weight gradient of a 3x3 / pad-1 stride-1 conv: dY / X fp32 through the bf16 pointer
// fields, Cs / Co in fp32 channels, standard taps; slab [splits][Co][9 Cs] fp32 as hwgrad
void hwgrad_f32(HWArgs a, int splits, hipStream_t s) {
  if (!hwgrad_f32_supported(a.NB, a.H, a.W, a.Cs, a.Co) || a.ntaps != 9)
    throw std::runtime_error("hwgrad_f32: unsupported shape");
  for (int t = 0; t < 9; ++t)
    if (a.tap_dy[t] != t / 3 - 1 || a.tap_dx[t] != t % 3 - 1) throw std::runtime_error("hwgrad_f32: 3x3 pad-1 taps only");
  if (splits != hwgrad_f32_splits(a.NB, a.H, a.W, a.Cs, a.Co)) throw std::runtime_error("hwgrad_f32: split count mismatch");
  // the bf16 view of the fp32 rows (see hwgrad2_kernel's F32 note)
  a.Cs *= 2; a.Co *= 2;
  a.npairs = 1; a.ldy = a.Co; a.ldx = a.Cs;
  a.pair_yoff[0] = a.pair_xoff[0] = 0; a.pair_bias[0] = 1;
  hw_geometry(a.H, a.W, &a.TH, &a.TW, &a.IMG);
  const int total = (a.NB / a.IMG) * (a.H / a.TH) * (a.W / a.TW);
  a.tiles_per_split = (total + splits - 1) / splits;
  const int grid = splits * (a.Co / 64) * (a.Cs / 64);
#define DCNN_HWF(TW_, TH_, IMG_, NS_)                                                                   \
  if (a.TW == TW_ && a.TH == TH_ && a.IMG == IMG_) {                                                    \
    auto k = hwgrad2_kernel<TW_, TH_, IMG_, NS_, 2, true>;                                              \
    const int lds = NS_ * HWGeo2<TW_, TH_, IMG_>::STAGE;                                                \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(grid, 1), dim3(512), lds, s, a);                                         \
    DCNN_LAUNCH_CHECK();                                                                                \
    return;                                                                                             \
  }
  DCNN_HWF(16, 8, 1, 3)
  DCNN_HWF(8, 8, 2, 2)
  DCNN_HWF(4, 4, 8, 2)
#undef DCNN_HWF
  throw std::runtime_error("hwgrad_f32: no kernel for this geometry");
}


// ---------------------------------------------------------------------------------------------
// Stride-2 halo weight gradient (3x3, pad 1, the downsampling convs of a ResNet stage):
//
//   dW[co][t][ci] = sum_p dY[p][co] * X[2 p + off_t][ci]
//
// A 64-pixel output tile (TW x TH x IMG) reaches a (2 TH + 1) x (2 TW + 1) input halo per image:
// staged once in LDS (natural row-major layout, zero-filled borders) and read by all 9 taps at a
// per-tap row offset dy * (2 TW + 1) + dx from the lane's pixel row 2 y + 1, 2 x + 1 — each lane
// of a transposing read supplies its own row address, so the stride needs no special layout. The
// gathered TN GEMM (gemm_t2) instead re-reads dY once per tap column block and gathers X per tap.
// 64-pixel tiles keep three (dY, halo) stages in LDS (48-52 KB each); the workgroup owns 64 (co)
// x 9 x 64 (ci) of dW as the stride-1 hwgrad_kernel, split-K slabs reduced by the caller.
// ---------------------------------------------------------------------------------------------
template <int TW, int TH, int IMG>
struct HWGeoS2 {
  static constexpr int TPX = TH * TW, PX = TPX * IMG;   // output pixels per tile (GEMM K)
  static constexpr int HW2 = 2 * TW + 1, HPI = (2 * TH + 1) * HW2, HP = IMG * HPI;
  static constexpr int HNI = (HP + 31) / 32;            // halo glds per wave per tile
  static constexpr int HPR = HNI * 32;
  static constexpr int YI = PX / 32;                    // dY glds per lane per tile
  static constexpr int KS = PX / 32;                    // 32-pixel k-steps per tile
  static constexpr int STAGE = PX * 128 + HPR * 128;
  static_assert(PX == 64, "64-pixel tiles");
};

// TSP = 2: 8 waves, two per SIMD — wave w + 4 shares wave w's 16 input channels and takes taps 5..8
// while wave w takes 0..4 (as hwgrad2_kernel); the first four waves issue the tile loads.
template <int TW, int TH, int IMG, int NS, int TSP = 1>
__global__ void __launch_bounds__(256 * TSP, 1) hwgrad_s2_kernel(HWArgs p) {
  prefetch_kernargs<sizeof(HWArgs)>();
  using G = HWGeoS2<TW, TH, IMG>;
  constexpr int HNI = G::HNI, HW2 = G::HW2, HPI = G::HPI, HP = G::HP, TPX = G::TPX, PX = G::PX;
  constexpr int YI = G::YI, KS = G::KS, STAGE = G::STAGE;
  constexpr int INS = YI + HNI;  // direct-to-LDS loads per lane per tile (the vmcnt unit)
  constexpr int ET = (NS * STAGE) / (64 * 68 * 4) < 9 ? (NS * STAGE) / (64 * 68 * 4) : 9;  // taps per epilogue pass
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = (tid >> 6) & 3, th = tid >> 8;
  constexpr int NT = 256 * TSP;
  const int co_tiles = p.Co / 64, ci_chunks = p.Cs / 64;
  const int per_split = co_tiles * ci_chunks;
  const int lt = xcd_remap_w(blockIdx.x, gridDim.x);
  const int split = lt / per_split, rem = lt - split * per_split;
  const int nsplits = gridDim.x / per_split;
  const int co0 = (rem / ci_chunks) * 64, c0 = (rem % ci_chunks) * 64;
  const int IH = 2 * p.H, IW = 2 * p.W;  // input grid (p.H x p.W is the output / dY grid)

  const int tx_tiles = p.W / TW, ty_tiles = p.H / TH, tpi = tx_tiles * ty_tiles;
  const int total_tiles = (p.NB / IMG) * tpi;
  const int tbeg = split * p.tiles_per_split;
  const int tend = min(total_tiles, tbeg + p.tiles_per_split);
  const i32x4 rsY = raw_rsrc(p.dY, p.dy_bytes);
  const i32x4 rsX = raw_rsrc(p.X, p.x_bytes);

  // ---- dY loader: YI glds per lane, rows (pixels) fixed relative to the tile origin ----
  const int slot = lane & 7;
  unsigned y_rel[YI], y_col[YI];
#pragma unroll
  for (int i = 0; i < YI; ++i) {
    const int row = (wid * YI + i) * 8 + (lane >> 3);
    const int im = row / TPX, r2 = row - im * TPX;
    y_rel[i] = (unsigned)((im * p.H + r2 / TW) * p.W + r2 % TW);
    y_col[i] = (unsigned)((co0 + ((slot ^ wswz(row)) * 8)) * 2);
  }
  // ---- halo loader: row (im, hy, hx) -> input pixel (2 y0 + hy, 2 x0 + hx), hy / hx from -1 ----
  int h_rel[HNI], h_hy[HNI], h_hx[HNI];
#pragma unroll
  for (int j = 0; j < HNI; ++j) {
    const int row = (wid * HNI + j) * 8 + (lane >> 3);
    const int im = row / HPI, r2 = row - im * HPI;
    const int hy = r2 / HW2 - 1, hx = r2 % HW2 - 1;
    const bool real = row < HP;
    h_hy[j] = real ? hy : -(1 << 20);  // padding rows of the buffer: never valid
    h_hx[j] = hx;
    h_rel[j] = ((im * IH + hy) * IW + hx) * p.Cs * 2 + (c0 + ((slot ^ wswz(row)) * 8)) * 2;
  }
  auto load_tile = [&](int buf, int tile) {
    if (TSP > 1 && th != 0) return;
    char* Ys = smem + buf * STAGE;
    char* Hs = Ys + PX * 128;
    const int ig = tile / tpi, tr = tile - ig * tpi;
    const int y0 = (tr / tx_tiles) * TH, x0 = (tr % tx_tiles) * TW;
    const int g0 = (ig * IMG * p.H + y0) * p.W + x0;  // tile origin pixel (dY grid)
#pragma unroll
    for (int i = 0; i < YI; ++i)
      glds16w(rsY, Ys + (wid * YI + i) * 1024, (unsigned)(g0 + y_rel[i]) * (unsigned)(p.Co * 2) + y_col[i]);
    const int gx = ((ig * IMG * IH + 2 * y0) * IW + 2 * x0) * p.Cs * 2;  // halo origin (input grid)
#pragma unroll
    for (int j = 0; j < HNI; ++j) {
      const bool ok = (unsigned)(2 * y0 + h_hy[j]) < (unsigned)IH && (unsigned)(2 * x0 + h_hx[j]) < (unsigned)IW;
      glds16w(rsX, Hs + (wid * HNI + j) * 1024, ok ? (unsigned)(gx + h_rel[j]) : kOOBw);
    }
  };

  // the first tile(s) go out before the halo-row table below (only ALU work until their waits)
  const int nt = tend - tbeg;
  if (nt > 0) load_tile(0, tbeg);
  if (NS == 3 && nt > 1) load_tile(1, tbeg + 1);

  // ---- per-lane halo row of the tap (0, 0) for each (k-step, half) pixel quad: input pixel
  //      (2 y + 1, 2 x + 1) of the halo for output pixel (y, x) ----
  int hrow[2 * KS];
#pragma unroll
  for (int s = 0; s < 2 * KS; ++s) {
    const int px = (s >> 1) * 32 + 8 * (lane >> 4) + (s & 1) * 4 + ((lane & 15) >> 2);
    const int im = px / TPX, r2 = px - im * TPX;
    hrow[s] = im * HPI + (2 * (r2 / TW) + 1) * HW2 + 2 * (r2 % TW) + 1;
  }

  auto run = [&](auto tb_c, auto ntw_c) {
  constexpr int TB = decltype(tb_c)::value, NTW = decltype(ntw_c)::value;
  f32x4 acc[4][NTW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int bcol = wid * 16 + 4 * (lane & 3);  // B column (input channel) this lane reads
  const bool do_bias = p.bias_slab != nullptr && c0 == 0 && th == 0;
  float bias_acc = 0.f;
  if (NS == 3 && nt > 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INS) : "memory");  // tile 0 landed, tile 1 may fly
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int it = 0; it < nt; ++it) {
    if (it + NS - 1 < nt) load_tile(cur == 0 ? NS - 1 : cur - 1, tbeg + it + NS - 1);
    const char* Ys = smem + cur * STAGE;
    const char* Hs = Ys + PX * 128;
    bf16x8 a[2][4], b[2][NTW];
    auto read_step = [&](int kk, bf16x8* av, bf16x8* bv) {
      const int krow = kk * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * (lane & 3);
        const bf16x4 lo = tr4(Ys, krow, col), hi = tr4(Ys, krow + 4, col);
        av[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int tl = 0; tl < NTW; ++tl) {
        const int t = TB + tl, toff = (t / 3 - 1) * HW2 + (t % 3 - 1);
        const bf16x4 lo = tr4(Hs, hrow[kk * 2] + toff, bcol), hi = tr4(Hs, hrow[kk * 2 + 1] + toff, bcol);
        bv[tl] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    read_step(0, a[0], b[0]);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int c = kk & 1;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): step kk's fragments have landed
      if (kk + 1 < KS) read_step(kk + 1, a[c ^ 1], b[c ^ 1]);
#pragma unroll
      for (int t = 0; t < NTW; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][i], b[c][t], acc[i][t], 0, 0, 0);
    }
    if (do_bias) {  // bias gradient: column sums of the staged dY tile (first ci chunk only)
      const int col = tid & 63, chn = col >> 3, w = (col & 7) * 2;
      for (int r = tid >> 6; r < PX; r += 4)
        bias_acc += (float)*reinterpret_cast<const bf16*>(Ys + r * 128 + ((chn ^ wswz(r)) << 4) + w);
    }
    if (NS == 3 && it + 2 < nt)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    cur = cur == NS - 1 ? 0 : cur + 1;
  }

  // ---- slab[split][co][t*Cs + ci] (as hwgrad_kernel) ----
  const long Ng = 9l * p.Cs;
  float* out = p.slab + (long)split * p.Co * Ng;
  float* stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int t0 = 0; t0 < 9; t0 += ET) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < ET; ++u) {
      const int tl = t0 + u - TB;  // this wave's accumulator slot of tap t0 + u
      if (t0 + u < 9 && tl >= 0 && tl < NTW) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(u * 64 + i * 16 + (lane >> 4) * 4 + r) * 68 + wid * 16 + (lane & 15)] = acc[i][tl][r];
      }
    }
    __syncthreads();
    const int nrows = (9 - t0 < ET ? 9 - t0 : ET) * 64;
    for (int q = tid; q < nrows * 16; q += NT) {
      const int row = q >> 4, c4 = (q & 15) * 4;
      const int u = row >> 6, co = co0 + (row & 63);
      const float4 v = *reinterpret_cast<const float4*>(stg + row * 68 + c4);
      *reinterpret_cast<float4*>(out + (long)co * Ng + (t0 + u) * p.Cs + c0 + c4) = v;
    }
  }
  if (p.bias_slab != nullptr && c0 == 0) {  // (every wave passes the same barriers)
    __syncthreads();
    if (tid < 256) stg[tid] = bias_acc;
    __syncthreads();
    if (tid < 64) p.bias_slab[(long)split * p.Co + co0 + tid] = stg[tid] + stg[tid + 64] + stg[tid + 128] + stg[tid + 192];
  }
  };
  // TSP == 2: the two wave groups run different instantiations of `run`, and both contain
  // workgroup barriers. They stay matched because every barrier in `run` sits in a loop or branch
  // whose bounds are workgroup-uniform and independent of the tap range (TB, NTW): the K loop over
  // this split's nt tiles, the epilogue's 9 / ET tap blocks, and the bias block (c0 == 0). Any
  // barrier added under a TB- or NTW-dependent condition would deadlock the workgroup; keep
  // tap-range dependence inside the barrier-free MFMA / staging code only.
  if constexpr (TSP == 1) {
    run(std::integral_constant<int, 0>{}, std::integral_constant<int, 9>{});
  } else {
    if (th == 0) run(std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{});
    else run(std::integral_constant<int, 5>{}, std::integral_constant<int, 4>{});
  }
  (void)nsplits;
}

// output-grid tile geometry of the stride-2 kernel: 8 x 8 tiles, or 4 x 4 maps four images a tile
static bool hw_s2_geometry(int H, int W, int* TH, int* TW, int* IMG) {
  if (H % 8 == 0 && W % 8 == 0) { *TW = 8; *TH = 8; *IMG = 1; return true; }
  if (H == 4 && W == 4) { *TW = 4; *TH = 4; *IMG = 4; return true; }
  return false;
}

bool hwgrad_s2_supported(int NB, int H, int W, int Cs, int Co) {
  int th, tw, img;
  if (Cs % 64 || Co % 64 || !hw_s2_geometry(H, W, &th, &tw, &img) || NB % img) return false;
  return (long)NB * 4 * H * W * Cs * 2 < (1l << 31) && (long)NB * H * W * Co * 2 < (1l << 31);
}

int hwgrad_s2_splits(int NB, int H, int W, int Cs, int Co) {
  int th, tw, img;
  if (!hw_s2_geometry(H, W, &th, &tw, &img)) return 1;
  const int total = (NB / img) * (H / th) * (W / tw);
  const int per_split = (Co / 64) * (Cs / 64);
  int want = (kHwTargetBlocks + per_split - 1) / per_split;
  if (want < 1) want = 1;
  constexpr int min_tps = 4;  // >= 256 pixels per split (64-pixel tiles)
  if (want > total / min_tps) want = total / min_tps > 1 ? total / min_tps : 1;
  const int tps = (total + want - 1) / want;
  return (total + tps - 1) / tps;
}

void hwgrad_s2(HWArgs a, int splits, hipStream_t s) {
  if (!hwgrad_s2_supported(a.NB, a.H, a.W, a.Cs, a.Co)) throw std::runtime_error("hwgrad_s2: unsupported shape");
  if (splits != hwgrad_s2_splits(a.NB, a.H, a.W, a.Cs, a.Co)) throw std::runtime_error("hwgrad_s2: split count mismatch");
  hw_s2_geometry(a.H, a.W, &a.TH, &a.TW, &a.IMG);
  const int total = (a.NB / a.IMG) * (a.H / a.TH) * (a.W / a.TW);
  a.tiles_per_split = (total + splits - 1) / splits;
  const int grid = splits * (a.Co / 64) * (a.Cs / 64);
#define DCNN_HWS2(TW_, TH_, IMG_)                                                                      \
  if (a.TW == TW_ && a.TH == TH_ && a.IMG == IMG_) {                                                   \
    auto k = hwgrad_s2_kernel<TW_, TH_, IMG_, 3, 2>;                                                   \
    const int lds = 3 * HWGeoS2<TW_, TH_, IMG_>::STAGE;                                                \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, s, a);                                           \
    DCNN_LAUNCH_CHECK();                                                                               \
    return;                                                                                            \
  }
  DCNN_HWS2(8, 8, 1)  // 3 x 48 KB
  DCNN_HWS2(4, 4, 4)  // 3 x 52 KB
#undef DCNN_HWS2
  throw std::runtime_error("hwgrad_s2: no variant");
}

}  // namespace dcnn
