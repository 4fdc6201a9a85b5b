// Third-generation halo-tiled 3x3 stride-1 convolution (forward and dgrad) for CDNA4:
// a persistent, cross-tile pipelined kernel.
//
// Work item = one 16 x 16 output pixel tile (an image window; on 8 x 8 / 4 x 4 maps a 2 x 2 /
// 4 x 4 grid of whole images separated by shared zero gutters) x 64 output channels and, on small
// grids, one split-K slice of its input channels. The grid is sized to the resident workgroups
// (2 per CU) and every workgroup walks its items in a strided order, so that:
//
//  * the next item's first halo chunk and first two weight stages are DMA'd into LDS during the
//    current item's last K steps (the (item, chunk, kernel-row) sequence is ONE stream: the halo
//    double buffer and the 2-stage weight ring never restart);
//  * the epilogue stores each 16-byte output row as soon as it is computed, AFTER issuing the
//    next item's second weight stage: the next item's first K step waits only for the loads
//    older than the stores, so the stores (and the statistics rows) drain under its MFMAs
//    instead of stalling the workgroup.
//
// Per item the structure is the round-3 one:
//
//  * 4 waves (256 threads), two workgroups per CU, each wave owning a 64 (output channels) x 64
//    (pixels) block: 16 accumulator tiles of mfma_f32_16x16x32_bf16.
//  * Weights are the A operand (rows = output channels), the input halo the B operand (columns =
//    pixels). The weight rows are loaded in a permuted channel order so that an accumulator
//    quad pair (i = 2h, 2h+1) holds 8 CONSECUTIVE channels of one pixel: the epilogue stores
//    16 bytes per lane, 64 contiguous bytes per pixel and wave instruction (8 dwordx4 stores per
//    lane instead of 16 dwordx2).
//  * K step = 32 input channels x one kernel row (3 taps): 48 MFMAs per wave per barrier. The
//    32-channel halo chunk (64-byte LDS rows) is loaded once per chunk and serves its 3 steps;
//    weights stream through a 2-stage ring with counted vmcnt waits and raw s_barrier
//    (direct-to-LDS loads stay in flight across barriers).
//  * Every LDS fragment address is precomputed (per-lane bases + immediates); halo source
//    addresses are decoded once per workgroup (pixel -> image / row / column of the halo) and
//    re-based per item with a handful of integer ops.
//  * Bank conflicts: 64-byte rows hold 4 16-byte chunks; pixel subtile row l carries pixel
//    perm(l) and the chunk is XOR-swizzled by bit 2 of the halo pixel index, so every 16-lane
//    ds_read_b128 group covers 16 distinct slots for any tap shift.
//
// fp32 instances (F32): IEEE fp32 operands on v_mfma_f32_16x16x4_f32 with the same LDS layout.
// A 16-channel fp32 chunk is 64 bytes per pixel, exactly a 32-channel bf16 chunk, so the launcher
// presents an fp32 tensor of C channels as a bf16 one of 2C (rows, taps, DMA pieces, swizzles and
// the tile plan unchanged); each 16-byte fragment is then 4 fp32 channels feeding 4 MFMAs (k = 4),
// the output and the residual are fp32 (HConvArgs::Cf / residual_f).
//
// Reference parity: the reference runs this GEMM as im2col + cuBLAS SGEMM or cuDNN
// (src/nn/layers_impl/cuda/conv2d_ops.cu:18-128, cudnn_conv2d_ops.cu:187-244).
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "api.h"
#include "hconv3_plan.h"

namespace dcnn {

namespace {
constexpr unsigned kOOB3 = 0x80000000u;

__device__ __forceinline__ int xcd_remap3(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// pixel carried by row l of a 16-pixel subtile, and the halo chunk swizzle (TWC: tile-width class)
template <int TWC>
__device__ __forceinline__ int h3_perm(int l) {
  if constexpr (TWC == 4) return l;
  return l < 4 ? l : (l >= 12 ? l - 8 : l + 4);
}
// (GUT: the 4 x 4-map gutter layout, runtime pitch 21: a 2-bit swizzle of pixel bits 2-3; the
// 1-bit one left 33% of its ds_read_b128 cycles bank-conflicted, profiles/pmc_stalls_r5.md)
template <int TWC, bool GUT = false>
__device__ __forceinline__ int h3_swz(int P) {
  if constexpr (GUT) return (P >> 2) & 3;
  if constexpr (TWC == 4) return ((P >> 3) & 1) << 1;
  return ((P >> 2) & 1) << 1;
}
__device__ __forceinline__ int h3_wswz(int n) { return ((n >> 3) & 1) << 1; }

// output channel (within the workgroup's BN) of weight-stage row n. Row m = 16 i + q of a wave's
// 64 is MFMA row q of accumulator tile i, which lands in lane group q >> 2, register q & 3; the
// channel 32 (i >> 1) + 8 (q >> 2) + 4 (i & 1) + (q & 3) gives lane group lh the 8 consecutive
// channels 32 h + 8 lh .. + 7 in tiles (2h, 2h+1)
__device__ __forceinline__ int h3_rowch(int n) {
  const int m = n & 63, i = m >> 4, q = m & 15;
  return (n & ~63) + 32 * (i >> 1) + 8 * (q >> 2) + 4 * (i & 1) + (q & 3);
}

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void h3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// fixed-order sum over the 16 lanes of a DPP row (rotations by 8 and 4, then quad swaps): every
// lane of the row gets the row total, with no LDS traffic
__device__ __forceinline__ float h3_row_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad xor 2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad xor 1
  return v;
}
// value of lane 0 of this lane's 16-lane DPP row (row_newbcast:0)
__device__ __forceinline__ float h3_row_first(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150, 0xf, 0xf, false));
}

template <int K, int N, class F>
__device__ __forceinline__ void h3_static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    h3_static_for<K + 1, N>(f);
  }
}

// direct-to-LDS 16-byte load to LDS byte address `base + OFF` (base: one wave-uniform SGPR for the
// whole kernel, OFF an immediate)
template <int OFF>
__device__ __forceinline__ void glds16_at(i32x4 rsrc, unsigned base, unsigned voff) {
  // (the operands are wave-uniform; readfirstlane pins them to SGPRs where the compiler's
  // divergence analysis loses track of that through the persistent loop's control flow)
  base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
  for (int i = 0; i < 4; ++i) rsrc[i] = __builtin_amdgcn_readfirstlane(rsrc[i]);
  asm volatile("s_add_u32 m0, %0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(base), "v"(voff), "s"(rsrc), "n"(OFF)
               : "memory", "m0");
}

__device__ __forceinline__ bf16x8 lds_b128(const char* smem, int off) {
  return *reinterpret_cast<const bf16x8*>(smem + off);
}
}  // namespace

// every lambda of the kernel is force-inlined: an outlined one receives its captures through a
// stack frame (scratch + flat loads of every captured register)
#define H3L __attribute__((always_inline))

// geometry the launcher computes once per call
// The output tile is TH x TW (16 x 16) pixels. Maps of 16 x 16 and larger: one image window
// (GY = GX = 1, IH = TH, IW = TW) at (y0, x0), its halo the neighbouring pixels. Smaller maps
// (8 x 8, 4 x 4): a GY x GX grid of whole IH x IW images side by side, separated by shared
// one-pixel zero gutters, so the halo is (TH + GY + 1) x (TW + GX + 1) with the same tap
// arithmetic (pixel (ty, tx) of the tile sits at halo (ty + ty / IH + 1, tx + tx / IW + 1)).
struct H3Geo {
  int TH, TW, pitch;       // spatial tile (16 x 16); halo row pitch (>= TW + GX + 1)
  int GY, GX, IH, IW;      // images per tile along y / x and their size (gutter layout if GY*GX > 1)
  int lGX, lIH, lIW;       // log2 of GX, IH, IW (powers of two)
  int tx_tiles, tpi;       // tiles per image row / per image group
  int tiles_n, tiles_m;    // channel tiles (N / BN), pixel tiles
  int nchunk;              // 32-channel chunks per split
  int nitems;              // tiles_m * tiles_n * splits
  int tb[9];               // weight column offset (elements) of tap (dy + 1) * 3 + (dx + 1)
  // the run-time divisors of the per-lane halo table as multiply-shift reciprocals (a plain
  // run-time division is a ~40-instruction sequence; the table did ~18 per lane)
  FastDiv fd_pitch, fd_ih1, fd_iw1;
  unsigned c_bytes;        // output bytes (32-bit store offsets)
  unsigned long long* stamps;  // diagnostic timeline [nitems][NW][16] (STAMP instance only)
};

// NW waves per workgroup, WC of them along the output channels (64 each), NW / WC along the
// pixels (64 each). PITCH > 0: compile-time halo row pitch (multiple of 8 pixels: a kernel-row
// shift keeps the chunk swizzle and becomes an immediate ds_read offset); 0: runtime pitch.
template <int NW, int WC, int TWC, int HN, int NWI, int PITCH>
struct H3 {
  static constexpr int BN = 64 * WC, WP = NW / WC, BM = 64 * WP;
  static constexpr int HALO = NW * HN * 1024;   // one halo buffer
  static constexpr int WST = NW * NWI * 1024;   // one weight stage (3 taps x BN rows x 64 B, padded)
  static constexpr int LDS = 2 * HALO + 2 * WST;
  static_assert(3 * BN * 64 <= WST, "weight stage");
  static_assert(WP * BN * 3 * 4 + 16 <= HALO, "epilogue scratch lives in the last chunk's halo buffer");
  static_assert(LDS <= 163840, "LDS budget");
};

// EPI: epilogue specialisation (compile-time: whether statistics rows are produced, and of which
// kind, is never a run-time branch): 0 = no statistics (bias / residual / ReLU at run time);
// 1 = forward BatchNorm statistics, no bias / residual / ReLU; 2 = data gradient with the
// backward-BatchNorm fusion (optional residual); 3 = forward statistics with bias / residual /
// ReLU at run time; 4 = EPI 2 with the ReLU mask recomputed from the BatchNorm input
// (BnbArgs::mask_x) instead of read from its output.
// STAMP: diagnostic instance with s_memtime stamps (benchmarks/hconv3_timeline.py).
template <int NW, int WC, int TWC, int HN, int NWI, int PITCH, int EPI, bool STAMP, bool F32 = false>
__global__ void __launch_bounds__(NW * 64, 8 / NW) hconv3_kernel(HConvArgs p, H3Geo g) {
  using T = H3<NW, WC, TWC, HN, NWI, PITCH>;
  constexpr int BN = T::BN, WP = T::WP;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  prefetch_kernargs<sizeof(HConvArgs) + sizeof(H3Geo) + 16>();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % WC, wp = wid / WC;
  const int lr = lane & 15, lh = lane >> 4;
  auto stamp = [&](int u, int k) H3L {
    if constexpr (STAMP) {
      if (lane == 0) g.stamps[((size_t)u * NW + wid) * 16 + k] = __builtin_amdgcn_s_memtime();
    }
  };
  const int SPL = p.splits;
  const int G = gridDim.x;
  int u = xcd_remap3(blockIdx.x, G);  // this workgroup's items: u, u + G, u + 2G, ...
  if (u >= g.nitems) return;          // (the launcher sizes the grid <= nitems)
  stamp(u, 5);
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += NT) p.zero_ptr[i] = 0.f;
  const i32x4 rsA = raw_rsrc(p.A, p.a_bytes);
  const i32x4 rsB = raw_rsrc(p.B, p.b_bytes);
  const int tx_tiles = g.tx_tiles, tpi = g.tpi;
  const int pitch = PITCH > 0 ? PITCH : g.pitch;
  const bool gut = g.GY * g.GX > 1;                     // gutter layout (whole small images)
  const int HW2 = g.TW + g.GX + 1;                       // halo columns
  const int HPX = (g.TH + g.GY + 1) * pitch;             // halo pixels per tile (pitch-padded)
  const int nch = g.nchunk;                              // chunks per item (even, or 1: a 32-channel input)
  stamp(u, 8);

  // ---- halo loader, item-invariant part (filled in the first item's prologue, after the first
  // weight DMA is issued: its latency hides the table's integer work)
  unsigned hpk[HN];
  // ---- weight loader, item-invariant part: stage row R = dx * BN + n (3 taps x BN rows, 64 B)
  unsigned wrc[NWI];  // (stage row's output channel + 1) | chunk slot byte offset << 16
  int wtb[NWI][3];  // byte offset of the instruction's tap column for kernel rows dy = 0..2 (SGPRs)
#pragma unroll
  for (int k = 0; k < NWI; ++k) {
    const int R0 = (wid * NWI + k) * 16;  // first stage row of the instruction (wave-uniform)
    const int R = R0 + (lane >> 2);
    const int dx = R0 / BN, n = R - dx * BN;
    // (a select over the three taps of the row, not a run-time index into the kernel arguments)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
      wtb[k][dy] = __builtin_amdgcn_readfirstlane(
          dx == 0 ? g.tb[dy * 3] * 2 : dx == 1 ? g.tb[dy * 3 + 1] * 2 : dx == 2 ? g.tb[dy * 3 + 2] * 2 : 0);
    wrc[k] = (unsigned)(dx < 3 ? h3_rowch(n) + 1 : 0) | ((unsigned)(((lane & 3) ^ h3_wswz(n)) * 16) << 16);
  }
  stamp(u, 10);

  // ---- per-item geometry and source addresses
  struct Item {
    int lt, zs, tm, n0, y0, x0, img0, cbase;
  };
  auto decode = [&](int v) H3L {
    Item t;
    t.zs = v % SPL;
    t.lt = v / SPL;
    t.tm = t.lt / g.tiles_n;
    t.n0 = (t.lt - t.tm * g.tiles_n) * BN;
    const int ig = t.tm / tpi, trem = t.tm - ig * tpi;
    t.y0 = (trem / tx_tiles) * 16;
    t.x0 = (trem % tx_tiles) * 16;
    t.img0 = ig * (g.GY * g.GX);
    t.cbase = t.zs * nch * 32;  // first input channel of this split
    return t;
  };
  auto addrs_h = [&](const Item& t, unsigned* hs) H3L {
#pragma unroll
    for (int k = 0; k < HN; ++k) {
      const unsigned pk = hpk[k];
      unsigned v = kOOB3;
      if (!(pk >> 31)) {
        const int sy = t.y0 + (int)((pk >> 8) & 255) - 1, sx = t.x0 + (int)(pk & 255) - 1;
        const int n = t.img0 + (int)((pk >> 16) & 255);
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W && n < p.NB)
          v = ((((unsigned)n * p.H + sy) * p.W + sx) * (unsigned)p.Cs + t.cbase + (pk >> 24) * 8) * 2u;
      }
      hs[k] = v;
    }
  };
  auto addrs_w = [&](const Item& t, unsigned* ws) H3L {
#pragma unroll
    for (int k = 0; k < NWI; ++k) {
      const int wr = (int)(wrc[k] & 0xffff) - 1;  // -1: padding row
      const int ch = t.n0 + wr;
      ws[k] = (wr >= 0 && ch < p.N) ? ((unsigned)ch * p.ldb + t.cbase) * 2u + (wrc[k] >> 16) : kOOB3;
    }
  };
  auto addrs = [&](const Item& t, unsigned* hs, unsigned* ws) H3L {
    addrs_h(t, hs);
    addrs_w(t, ws);
  };

  // LDS byte address of this wave's first halo / weight DMA slot (wave-uniform SGPRs)
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)smem));
  const unsigned hbase = lds0 + wid * HN * 1024, wbase_lds = lds0 + 2 * T::HALO + wid * NWI * 1024;
  auto load_halo = [&](auto buf_c, int c, const unsigned* hs) H3L {
    constexpr int BUF = decltype(buf_c)::value;
    const unsigned co = (unsigned)(c * 64);
    h3_static_for<0, HN>([&](auto kc) H3L {
      constexpr int K = decltype(kc)::value;
      glds16_at<BUF * T::HALO + K * 1024>(rsA, hbase, hs[K] + co);
    });
  };
  auto load_w = [&](auto stage_c, int c, int dy, const unsigned* ws) H3L {
    constexpr int ST = decltype(stage_c)::value;
    h3_static_for<0, NWI>([&](auto kc) H3L {
      constexpr int K = decltype(kc)::value;
      glds16_at<ST * T::WST + K * 1024>(rsB, wbase_lds, ws[K] + (unsigned)(wtb[K][dy] + c * 64));
    });
  };

  // ---- fragment addresses
  // A (weights): row n = wc*64 + i*16 + lr of stage tap dx: stage + dx*BN*64 + (wc*64 + i*16)*64 + abase
  const int abase = 2 * T::HALO + (wc * 64 + lr) * 64 + ((lh ^ h3_wswz(lr)) << 4);
  // B (halo): pixel subtile j of this wave, tap (dy, dx)
  constexpr int NBA = PITCH > 0 ? 3 : 9;
  static_assert(PITCH == 0 || (PITCH % 8 == 0 && TWC != 4), "dy-invariant swizzle needs pitch % 8 == 0");
  // (re-derived at the start of every item from an opaque zero, so the 4 x NBA addresses are not
  // kept live through the epilogue, where the persistent loop has no registers to spare)
  int baddr[4][NBA];
  auto set_baddr = [&](int zero) H3L {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = wp * 64 + j * 16 + h3_perm<TWC>(lr);  // tile-local output pixel
      const int ty = q >> 4, tx = q & 15;  // (16 x 16 tiles)
      // halo pixel of tap (-1, -1) (gutter layout: one gutter row / column per image crossed)
      const int P0 = (ty + (ty >> g.lIH)) * pitch + tx + (tx >> g.lIW) + zero;
#pragma unroll
      for (int t = 0; t < NBA; ++t) {
        const int P = P0 + (NBA == 3 ? t : (t / 3) * pitch + (t % 3));
        baddr[j][t] = P * 64 + ((lh ^ h3_swz<TWC, HN == 7>(P)) << 4);
      }
    }
  };

  auto baddr_of = [&](int j, int dy, int dx) H3L {
    if constexpr (PITCH > 0) return baddr[j][dx] + dy * PITCH * 64;
    else return baddr[j][dy * 3 + dx];
  };
  // output row offsets (bytes, first channel of the lane group) of the tile's pixel subtiles
  auto out_offsets = [&](const Item& t, unsigned* oo) H3L {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = wp * 64 + j * 16 + h3_perm<TWC>(lr);
      const int ty = q >> 4, tx = q & 15;
      const int iy = ty >> g.lIH, ix = tx >> g.lIW;  // (0, 0) unless gutter layout
      const unsigned pix = ((unsigned)(t.img0 + (iy << g.lGX) + ix) * p.H + t.y0 + ty - (iy << g.lIH)) * p.W + t.x0 +
                           tx - (ix << g.lIW);
      oo[j] = (pix * (unsigned)p.N + t.n0 + wc * 64 + 8 * lh) * (F32 ? 4u : 2u);
    }
  };

  f32x4 acc[4][4];
  // one K step: chunk c (halo buffer HB), kernel row DY, weight stage ST. The fragments of tap
  // dx + 1 are read while tap dx's 16 MFMAs run, so the LDS latency after the barrier is paid
  // once per step. The step's direct-to-LDS loads and deferred stores (`issue`) go out after the
  // first MFMAs.
  auto step = [&](auto hb_c, auto dy_c, auto st_c, auto pre, auto issue) H3L {
    constexpr int HB = decltype(hb_c)::value, DY = decltype(dy_c)::value, ST = decltype(st_c)::value;
    bf16x8 a[3][4], b[3][4];
    auto rd = [&](int dx) H3L {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[dx][i] = lds_b128(smem, abase + ST * T::WST + dx * BN * 64 + i * 16 * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[dx][j] = lds_b128(smem, baddr_of(j, DY, dx) + HB * T::HALO);
    };
    auto mm = [&](int dx, int i0, int i1) H3L {
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F32) {
        // 4 fp32 channels per fragment lane: lane group lh holds channels 4 lh .. 4 lh + 3 of the
        // chunk, MFMA m takes channel 4 lh + m as its k = lh (A and B alike), the 4 MFMAs of a tile
        // are 16 independent MFMAs apart
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int i = i0; i < i1; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x4 av = __builtin_bit_cast(f32x4, a[dx][i]), bv = __builtin_bit_cast(f32x4, b[dx][j]);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[m], acc[i][j], 0, 0, 0);
            }
      } else {
#pragma unroll
        for (int i = i0; i < i1; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[dx][i], b[dx][j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
    };
    pre();
    rd(0);
    rd(1);
    mm(0, 0, 2);
    issue();
    mm(0, 2, 4);
    rd(2);
    mm(1, 0, 4);
    mm(2, 0, 4);
  };

  unsigned oo[4];  // output row offsets of the item's pixel subtiles
  char* const cbytes = reinterpret_cast<char*>(p.C);
  auto nothing = []() H3L {};

  // ---- first item's prologue: halo chunk 0, W(0, 0) landed; W(0, 1) in flight
  auto fill_hpk = [&]() H3L {
    // ---- halo loader, item-invariant part: instruction k of this wave fills halo pixels
    // [16(wid*HN + k), +16); lane -> (image, row + 1, column + 1 within the image window, chunk
    // slot), packed; gutters and row padding are never loaded (zero-filled by the buffer range)
#pragma unroll
    for (int k = 0; k < HN; ++k) {
      const int P = (wid * HN + k) * 16 + (lane >> 2);
      unsigned v = 0xffffffffu;
      if (P < HPX) {
        const int hy = (int)fdiv((unsigned)P, g.fd_pitch), hx = P - hy * pitch;
        int cy = hy, cx = hx, im = 0;
        bool ok = hx < HW2;
        if (gut) {
          const int iy = (int)fdiv((unsigned)hy, g.fd_ih1), ix = (int)fdiv((unsigned)hx, g.fd_iw1);
          cy = hy - iy * (g.IH + 1);
          cx = hx - ix * (g.IW + 1);
          im = iy * g.GX + ix;
          ok = ok && cy != 0 && cx != 0;
        }
        if (ok) v = (unsigned)cx | ((unsigned)cy << 8) | ((unsigned)im << 16) | ((unsigned)((lane & 3) ^ h3_swz<TWC, HN == 7>(P)) << 24);
      }
      hpk[k] = v;
    }
  };
  unsigned hs[HN], ws[NWI];
  const Item t0 = decode(u);
  if constexpr (HN != 7) {
    // (issue order W(0, 0), halo chunk 0, W(0, 1): the weight DMA goes out before the halo table
    // is built and the fragment addresses are derived while both are in flight; vmcnt(NWI) below
    // still means "W(0, 0) and the halo landed, W(0, 1) in flight")
    addrs_w(t0, ws);
    load_w(I0{}, 0, 0, ws);
    fill_hpk();
    stamp(u, 9);
    addrs_h(t0, hs);
    stamp(u, 6);
    load_halo(I0{}, 0, hs);
    load_w(I1{}, 0, 1, ws);
    set_baddr(0);
    stamp(u, 11);
  } else {
    // (the 4 x 4-map gutter instances keep the plain order: the one above spills VGPRs there)
    fill_hpk();
    stamp(u, 9);
    set_baddr(0);
    stamp(u, 11);
    addrs(t0, hs, ws);
    stamp(u, 6);
    load_halo(I0{}, 0, hs);
    load_w(I0{}, 0, 0, ws);
    load_w(I1{}, 0, 1, ws);
  }
  vmwait<NWI>();
  stamp(u, 7);
  h3_barrier();
  int nst = 0;  // output stores issued after the item's W(0, 1) (the previous item's epilogue)

  while (true) {
    stamp(u, 0);

    const int un = u + G;
    const bool has_next = un < g.nitems;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // 2-stage ring: step s uses stage s & 1 = (chunk + dy) & 1 (3 steps per chunk) = the chunk's
    // halo buffer at dy = 0. Step (c, 0) issues W(c, 1) and the next halo chunk (this item's
    // c + 1, or the next item's chunk 0); step (c, 1) issues W(c, 2); step (c, 2) issues the next
    // chunk's W(., 0) (this item's, or the next item's). The wait after a step retires that step's
    // weights and the halo issued before it. In the last chunk the next item's source addresses
    // replace this item's (halo after step 0's issue, weights after step 1's), so no second set
    // of address registers stays live.
    // Item boundary: the next item's W(0, 1) goes out at the start of this item's epilogue (its
    // stage is free once the last step's barrier has passed), BEFORE the epilogue's output stores.
    // So the first step of the next item does not issue W(0, 1) and its wait leaves the stores in
    // flight: they drain under that step's MFMAs instead of stalling the workgroup.
    auto chunk = [&](int c, auto hb_c, auto first_c) H3L {
      constexpr int HB = decltype(hb_c)::value;
      constexpr bool FIRST = decltype(first_c)::value;
      using S0 = std::integral_constant<int, HB>;
      using S1 = std::integral_constant<int, HB ^ 1>;
      const bool last = c + 1 == nch;
      const bool more = !last || has_next;
      auto dma0 = [&]() H3L {
        if constexpr (!FIRST) load_w(S1{}, c, 1, ws);
        if (!last) {
          load_halo(S1{}, c + 1, hs);
        } else if (has_next) {
          addrs_h(decode(un), hs);
          load_halo(S1{}, 0, hs);
        }
      };
      step(hb_c, I0{}, S0{}, nothing, dma0);
      if constexpr (FIRST) {
        // W(c, 1) is older than the stores and the halo
        if (nst) {
          if (more) vmwait<HN + 8>(); else vmwait<8>();
        } else {
          if (more) vmwait<HN>(); else vmwait<0>();
        }
      } else {
        if (more) vmwait<HN>(); else vmwait<0>();
      }
      h3_barrier();
      step(hb_c, I1{}, S1{}, nothing, [&]() H3L { load_w(S0{}, c, 2, ws); });
      vmwait<0>();
      h3_barrier();
      step(hb_c, I2{}, S0{}, nothing, [&]() H3L {
        if (!last) {
          load_w(S1{}, c + 1, 0, ws);
        } else if (has_next) {
          addrs_w(decode(un), ws);
          load_w(S1{}, 0, 0, ws);
        }
      });
      vmwait<0>();
      h3_barrier();
    };
    auto kloop = [&](auto h0_c) H3L {
      constexpr int H0 = decltype(h0_c)::value;
      using F = std::integral_constant<bool, false>;
      chunk(0, std::integral_constant<int, H0>{}, std::integral_constant<bool, true>{});
      stamp(u, 1);
      for (int c = 1; c < nch; c += 2) {
        chunk(c, std::integral_constant<int, H0 ^ 1>{}, F{});
        if (c + 1 < nch) chunk(c + 1, std::integral_constant<int, H0>{}, F{});
      }
    };
    kloop(I0{});
    stamp(u, 2);
    nst = 0;
    const int hb_last = (nch - 1) & 1;  // (nch even, or one item per workgroup)
    // the next item's W(0, 1) into the stage the last step read (ws holds the next item's weight
    // addresses since the last step's issue)
    if (has_next) {
      if (hb_last) load_w(I1{}, 0, 1, ws); else load_w(I0{}, 0, 1, ws);
    }
    // epilogue scratch: the last chunk's halo buffer, free until the next item's first step issues
    // its second halo chunk into it (after the closing barrier below)
    float* red = reinterpret_cast<float*>(smem + hb_last * T::HALO);
    volatile int* flag = reinterpret_cast<volatile int*>(smem + hb_last * T::HALO + WP * BN * 12);

    const Item it = decode(u);
    bool run_epi = true;
    // ---------------------------------------------------------------- split-K hand-off
    if (SPL > 1) {
      // every partial leaves with agent-scope (sc1) 16-byte buffer stores ([split][tile i, j][lane]
      // per output tile: one 4 KB row per instruction), each wave drains them, one lane adds to the
      // tile's ticket behind the workgroup barrier, and the workgroup whose add returns SPL - 1
      // reads the partials back with sc1 loads (16 in flight per split) and sums them in split order
      const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc(
          p.part + (size_t)it.lt * SPL * 16 * NT * 4, 0, SPL * 16 * NT * 16, 0x00020000);
      constexpr int kSC1 = 16;  // cache policy: sc1 (agent-coherent)
      using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsP,
                                                 ((it.zs * 16 + i * 4 + j) * NT + tid) * 16, 0, kSC1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(p.tickets + it.lt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int lst = old == (unsigned)(SPL - 1);
        if (lst) __hip_atomic_store(p.tickets + it.lt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = lst;
      }
      __syncthreads();
      run_epi = __builtin_amdgcn_readfirstlane(*flag) != 0;  // (uniform: keeps the DMA operands in SGPRs)
      __syncthreads();
      if (run_epi) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < SPL; ++z) {
          f32x4 t[16];
#pragma unroll
          for (int k = 0; k < 16; ++k)
            t[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsP, ((z * 16 + k) * NT + tid) * 16, 0, kSC1));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += t[i * 4 + j];
        }
      }
    }

    if (run_epi) {
      // -------------------------------------------------------------- epilogue (from registers)
      // lane (lh, lr): pixel subtile j -> tile pixel wp*64 + j*16 + perm(lr); channel half h ->
      // channels cb + 32 h + e (e = 0..7) = acc[2h + (e >> 2)][j][e & 3], cb = n0 + wc*64 + 8*lh.
      // Per channel half: operand loads (bias, BN mean / istd, residual, ReLU output, BN input),
      // arithmetic, 4 x 16-byte stores, statistics rows.
      constexpr bool bnb = EPI == 2 || EPI == 4, stats = EPI != 0, opts = EPI == 0 || EPI == 3;
      constexpr bool mask_x = EPI == 4;  // (the ReLU mask recomputed from x: BnbArgs::mask_x)
      const bool has_res = EPI != 1 && p.residual != nullptr, has_y = EPI == 2 && p.bnb.y != nullptr;
      constexpr bool has_x = bnb;
      const bool has_bias = opts && p.bias != nullptr, relu = opts && p.relu;
      const int cb = it.n0 + wc * 64 + 8 * lh;
      out_offsets(it, oo);
      const char* rbytes = reinterpret_cast<const char*>(p.residual);
      const char* ybytes = reinterpret_cast<const char*>(p.bnb.y);
      const char* xbytes = reinterpret_cast<const char*>(p.bnb.x);
      // one channel half at a time (keeps the epilogue's operand registers to a half)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (it.n0 + wc * 64 + 32 * h >= p.N) continue;  // (wave-uniform: the N = 32 tile's upper half)
        float bv[8], mu[8], is[8], msc[8], msf[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bv[e] = has_bias ? p.bias[cb + 32 * h + e] : 0.f;
          mu[e] = has_x ? p.bnb.mean[cb + 32 * h + e] : 0.f;
          is[e] = has_x ? p.bnb.istd[cb + 32 * h + e] : 0.f;
        }
        if constexpr (!F32 && mask_x) {  // the forward apply's scale / shift, same expressions
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gm = p.bnb.gamma ? p.bnb.gamma[cb + 32 * h + e] : 1.f;
            const float bt = p.bnb.beta ? p.bnb.beta[cb + 32 * h + e] : 0.f;
            msc[e] = gm * is[e];
            msf[e] = bt - mu[e] * gm * is[e];
          }
        }
        float gv[4][8], xh[4][8];  // [j][e]: stored value, and (bnb) stored value * xhat
        if constexpr (F32) {
          // fp32 output (+ fp32 residual): 32 bytes per lane and channel half; with the
          // backward-BatchNorm fusion (EPI 2) the consuming BatchNorm's fp32 ReLU output (mask) and
          // input (xhat) come in the same 32-byte rows
          const char* rfb = reinterpret_cast<const char*>(p.residual_f);
          char* cfb = reinterpret_cast<char*>(p.Cf);
          const bool has_rf = p.residual_f != nullptr;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const unsigned o = oo[j] + h * 128;
            float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0;
            if (has_rf) {
              r0 = *reinterpret_cast<const float4*>(rfb + o);
              r1 = *reinterpret_cast<const float4*>(rfb + o + 16);
            }
            const float rf[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
            if constexpr (bnb) {
              float4 y0 = make_float4(1.f, 1.f, 1.f, 1.f), y1 = y0;
              if (has_y) {
                y0 = *reinterpret_cast<const float4*>(ybytes + o);
                y1 = *reinterpret_cast<const float4*>(ybytes + o + 16);
              }
              const float4 x0 = *reinterpret_cast<const float4*>(xbytes + o);
              const float4 x1 = *reinterpret_cast<const float4*>(xbytes + o + 16);
              const float yf[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
              const float xf[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                float f = acc[2 * h + (e >> 2)][j][e & 3];
                if (has_rf) f += rf[e];
                f = yf[e] > 0.f ? f : 0.f;
                gv[j][e] = f;
                xh[j][e] = f * ((xf[e] - mu[e]) * is[e]);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                float f = acc[2 * h + (e >> 2)][j][e & 3] + bv[e];
                if (has_rf) f += rf[e];
                if (relu) f = fmaxf(f, 0.f);
                gv[j][e] = f;
                xh[j][e] = 0.f;
              }
            }
            *reinterpret_cast<float4*>(cfb + o) = make_float4(gv[j][0], gv[j][1], gv[j][2], gv[j][3]);
            *reinterpret_cast<float4*>(cfb + o + 16) = make_float4(gv[j][4], gv[j][5], gv[j][6], gv[j][7]);
          }
        } else {
        uint4 rr[4], yy[4], xx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned o = oo[j] + h * 64;
          rr[j] = has_res ? *reinterpret_cast<const uint4*>(rbytes + o) : make_uint4(0u, 0u, 0u, 0u);
          yy[j] = has_y ? *reinterpret_cast<const uint4*>(ybytes + o) : make_uint4(0u, 0u, 0u, 0u);
          xx[j] = has_x ? *reinterpret_cast<const uint4*>(xbytes + o) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float f[8], rf[8], yf[8], xf[8];
          unpack8(rr[j], rf);
          unpack8(yy[j], yf);
          unpack8(xx[j], xf);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            f[e] = acc[2 * h + (e >> 2)][j][e & 3] + bv[e];
            if (has_res) f[e] += rf[e];
            if (relu) f[e] = fmaxf(f[e], 0.f);
            if (has_y) f[e] = yf[e] > 0.f ? f[e] : 0.f;
            if constexpr (mask_x) f[e] = xf[e] * msc[e] + msf[e] > 0.f ? f[e] : 0.f;
          }
          const uint4 ov = pack8(f);
          *reinterpret_cast<uint4*>(cbytes + oo[j] + h * 64) = ov;
          unpack8(ov, gv[j]);  // statistics of the values actually stored
#pragma unroll
          for (int e = 0; e < 8; ++e) xh[j][e] = has_x ? gv[j][e] * ((xf[e] - mu[e]) * is[e]) : 0.f;
        }
        }
        if (stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float pv, sa, sb;
            if (bnb) {
              pv = 0.f;
              sa = (gv[0][e] + gv[1][e]) + (gv[2][e] + gv[3][e]);
              sb = (xh[0][e] + xh[1][e]) + (xh[2][e] + xh[3][e]);
            } else {
              // forward Welford rows: sums about a pivot (the wave's first pixel of the channel:
              // lane 16*lh of the DPP row)
              pv = h3_row_first(gv[0][e]);
              float a = 0.f, b = 0.f;
#pragma unroll
              for (int j = 0; j < 4; ++j) { const float d = gv[j][e] - pv; a += d; b += d * d; }
              sa = a;
              sb = b;
            }
            sa = h3_row_sum(sa);  // fixed-order sum over the 16 lanes (pixels) of the DPP row
            sb = h3_row_sum(sb);
            if (lr == 0) {
              float* q = red + (wp * BN + wc * 64 + 32 * h + 8 * lh + e) * 3;
              q[0] = pv;
              q[1] = sa;
              q[2] = sb;
            }
          }
        }
      }
      nst = 8;
      stamp(u, 3);
      if (stats) {
        __syncthreads();
        if (tid < BN && it.n0 + tid < p.N) {
          if (bnb) {
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int w = 0; w < WP; ++w) { a += red[(w * BN + tid) * 3 + 1]; b += red[(w * BN + tid) * 3 + 2]; }
            p.stats[((long)it.tm * 2 + 0) * p.N + it.n0 + tid] = a;
            p.stats[((long)it.tm * 2 + 1) * p.N + it.n0 + tid] = b;
          } else {
            Welford w = welford_from_shifted(64.f, red[tid * 3 + 0], red[tid * 3 + 1], red[tid * 3 + 2]);
#pragma unroll
            for (int k = 1; k < WP; ++k) {
              const float* e = red + (k * BN + tid) * 3;
              w = welford_merge(w, welford_from_shifted(64.f, e[0], e[1], e[2]));
            }
            store_welford(p.stats, it.tm, p.N, it.n0 + tid, w);
          }
        }
        // the scratch stage is the next item's first DMA target
        __syncthreads();
      }
    }
    stamp(u, 4);
    if (!has_next) break;
    u = un;
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
int hconv_split_target();  // hconv.hip (hconv_set_split_target; 0 = never split)

static int g_h3 = 1;  // hconv3_enable(0): the previous kernel (test hook)
void hconv3_enable(int on) { g_h3 = on; }
static unsigned long long* g_h3_stamps = nullptr;
void hconv3_set_stamps(uintptr_t p) { g_h3_stamps = reinterpret_cast<unsigned long long*>(p); }
static int g_h3_grid_cap = 0;  // test hook: at most this many persistent workgroups (0: resident count)
void hconv3_set_grid_cap(int n) { g_h3_grid_cap = n < 0 ? 0 : n; }
static int g_h3_max_splits = 8;  // tuning hook: split-K slices per tile at most
void hconv3_set_max_splits(int n) { g_h3_max_splits = n < 1 ? 1 : n; }

// tile plan for a 3x3 stride-1 conv of NB x H x W pixels, Cs input / N output channels
bool hconv3_plan(int NB, int H, int W, int Cs, int N, int ntaps, H3Plan* pl) {
  // an even 32-channel chunk count (split-K pairs), or one chunk (32 input channels: ResNet-18's
  // first residual conv)
  // N = 32 (the 32-channel data gradient of ResNet-18's first residual conv): one 64-channel tile
  // whose upper half reads zero weights (buffer range) and is neither stored nor counted
  if (!g_h3 || ntaps != 9 || (Cs % 64 && Cs != 32) || (N % 64 && N != 32)) return false;
  // 4-wave workgroups of 64 output channels x one 16 x 16 pixel tile, two per CU. Maps of 16 x 16
  // and larger (multiples of 16): image windows, halo 18 x 18 (pitch 18, 6 DMA instructions per
  // wave and chunk, LDS 72 KB). 8 x 8 maps: 2 x 2 images per tile, halo 19 x 19 (6 instructions);
  // 4 x 4 maps: 4 x 4 images, halo 21 x 21 (7 instructions, LDS 80 KB).
  constexpr int NW = 4, BN = 64, TH = 16, TW = 16;
  int GY = 1, GX = 1;
  if (H == 8 && W == 8) GY = GX = 2;
  else if (H == 4 && W == 4) GY = GX = 4;
  else if (H % TH || W % TW) return false;
  if (NB % (GY * GX)) return false;
  pl->TH = TH; pl->TW = TW; pl->GY = GY; pl->GX = GX;
  pl->IH = GY > 1 ? H : TH;
  pl->IW = GX > 1 ? W : TW;
  pl->pitch = TW + GX + 1;
  pl->HN = ((TH + GY + 1) * pl->pitch + 16 * NW - 1) / (16 * NW);
  if (pl->HN != 6 && pl->HN != 7) return false;  // the compiled instances
  pl->tx_tiles = GX > 1 ? 1 : W / TW;
  pl->tpi = GX > 1 ? 1 : (W / TW) * (H / TH);
  pl->tiles_m = NB * H * W / (TH * TW);
  pl->tiles_n = (N + BN - 1) / BN;
  // split-K over 32-channel chunks until the work items reach the target count (hconv.hip
  // g_split_target: one per CU); a split may hold a single chunk (then every workgroup runs one
  // item), at most 8 splits (the last arriver reads every partial back)
  const long tiles = (long)pl->tiles_m * pl->tiles_n;
  const int nchunk = Cs / 32, target = hconv_split_target();
  int s = 1;
  while (tiles * s < target && nchunk % (2 * s) == 0 && s < g_h3_max_splits) s *= 2;
  pl->splits = s;
  return true;
}

template <int NW, int WC, int TWC, int HN, int NWI, int PITCH, int EPI, bool STAMP, bool F32 = false>
static void launch_h3e(const HConvArgs& a, const H3Geo& g, hipStream_t s) {
  using T = H3<NW, WC, TWC, HN, NWI, PITCH>;
  auto k = hconv3_kernel<NW, WC, TWC, HN, NWI, PITCH, EPI, STAMP, F32>;
  constexpr int lds = T::LDS;
  static int resident = 0;  // workgroups of this instance the device holds at once
  if (!resident) {
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    int dev = 0, cus = 0, per_cu = 0;
    DCNN_HIP_CHECK(hipGetDevice(&dev));
    DCNN_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DCNN_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, NW * 64, lds));
    resident = cus * (per_cu > 0 ? per_cu : 1);
  }
  // persistent grid: at most the resident workgroups, items spread evenly (every workgroup walks
  // ceil or floor of nitems / grid items)
  int grid = g.nitems < resident ? g.nitems : resident;
  if (g_h3_grid_cap > 0 && grid > g_h3_grid_cap) grid = g_h3_grid_cap;
  // an odd chunk count (one 32-channel chunk) would alternate the halo buffer parity from item to
  // item; the kernel is compiled for items starting in buffer 0, so those run one item each
  if (g.nchunk & 1) grid = g.nitems;
  const int per = (g.nitems + grid - 1) / grid;
  grid = (g.nitems + per - 1) / per;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, s, a, g);
  DCNN_LAUNCH_CHECK();
}

// the epilogue instance for these options (-1: not covered)
static int h3_epi(const HConvArgs& a) {
  if (a.bnb.x) return (a.stats && !a.relu && !a.bias) ? (a.bnb.mask_x && !a.Cf ? 4 : 2) : -1;
  if (!a.stats) return 0;
  return (a.residual || a.residual_f || a.relu || a.bias) ? 3 : 1;
}

template <int NW, int WC, int TWC, int HN, int NWI, int PITCH>
static void launch_h3(const HConvArgs& a, const H3Geo& g, hipStream_t s) {
  const int epi = h3_epi(a);
  if (a.Cf) {  // fp32 operands (hconv3_f32_try)
    if (epi == 1) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 1, false, true>(a, g, s);
    if (epi == 2) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 2, false, true>(a, g, s);
    if (epi == 3) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 3, false, true>(a, g, s);
    return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 0, false, true>(a, g, s);
  }
  // (timeline instances: the statistics forward and the plain dgrad)
  if (g.stamps && epi == 1) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 1, true>(a, g, s);
  if (g.stamps && epi == 0) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 0, true>(a, g, s);
  if (epi == 1) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 1, false>(a, g, s);
  if (epi == 2) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 2, false>(a, g, s);
  if (epi == 3) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 3, false>(a, g, s);
  if (epi == 4) return launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 4, false>(a, g, s);
  launch_h3e<NW, WC, TWC, HN, NWI, PITCH, 0, false>(a, g, s);
}

static void launch_h3_plan(const H3Plan& pl, const HConvArgs& a, const H3Geo& g, hipStream_t s) {
  if (pl.HN == 6) return launch_h3<4, 1, 16, 6, 3, 0>(a, g, s);
  if (pl.HN == 7) return launch_h3<4, 1, 16, 7, 3, 0>(a, g, s);
  throw std::runtime_error("hconv3: no kernel instance for this plan");
}

static bool hconv3_run(const HConvArgs& a0, hipStream_t s);

// returns false when the shape / taps / epilogue options are not covered (caller falls back)
bool hconv3_try(const HConvArgs& a0, hipStream_t s) {
  if (a0.Cf) return false;
  return hconv3_run(a0, s);
}

// fp32 operands: A / B fp32 (passed through the bf16 pointer fields), Cs fp32 input channels,
// ldb / tap_b in fp32 elements, output Cf (+ residual_f), no backward-BN fusion. Presented to the
// plan as bf16 with 2 Cs channels (see the header comment).
bool hconv3_f32_try(const HConvArgs& a0, hipStream_t s) {
  if (!a0.Cf || a0.residual) return false;  // (bnb.y / bnb.x: fp32 tensors through the bf16 fields)
  HConvArgs a = a0;
  a.Cs = 2 * a0.Cs;
  a.ldb = 2 * a0.ldb;
  for (int t = 0; t < a.ntaps; ++t) a.tap_b[t] = 2 * a0.tap_b[t];
  if ((long)a.NB * a.H * a.W * a.N * 4 >= 0x80000000l) return false;
  return hconv3_run(a, s);
}

int hconv3_f32_splits(int NB, int H, int W, int Cs, int N, int ntaps) {
  H3Plan pl;
  return hconv3_plan(NB, H, W, 2 * Cs, N, ntaps, &pl) ? pl.splits : 0;
}

static bool hconv3_run(const HConvArgs& a0, hipStream_t s) {
  H3Plan pl;
  if (h3_epi(a0) < 0 || !hconv3_plan(a0.NB, a0.H, a0.W, a0.Cs, a0.N, a0.ntaps, &pl)) return false;
  H3Geo g{};
  for (int t = 0; t < 9; ++t) g.tb[t] = -1;
  for (int t = 0; t < a0.ntaps; ++t) {
    const int dy = a0.tap_dy[t], dx = a0.tap_dx[t];
    if (dy < -1 || dy > 1 || dx < -1 || dx > 1) return false;
    g.tb[(dy + 1) * 3 + dx + 1] = a0.tap_b[t];
  }
  for (int t = 0; t < 9; ++t)
    if (g.tb[t] < 0) return false;
  const long c_bytes = (long)a0.NB * a0.H * a0.W * a0.N * (a0.Cf ? 4 : 2);
  if (a0.a_bytes >= 0x80000000u || a0.b_bytes >= 0x80000000u || c_bytes >= 0x80000000l) return false;
  HConvArgs a = a0;
  if (a.splits != pl.splits) throw std::runtime_error("hconv3: split count mismatch (use hconv_splits)");
  if (pl.splits > 1 && (!a.part || !a.tickets)) throw std::runtime_error("hconv3: split-K workspace missing");
  g.TH = pl.TH; g.TW = pl.TW; g.pitch = pl.pitch;
  g.GY = pl.GY; g.GX = pl.GX; g.IH = pl.IH; g.IW = pl.IW;
  g.lGX = __builtin_ctz(pl.GX); g.lIH = __builtin_ctz(pl.IH); g.lIW = __builtin_ctz(pl.IW);
  g.tx_tiles = pl.tx_tiles; g.tpi = pl.tpi;
  g.tiles_n = pl.tiles_n; g.tiles_m = pl.tiles_m;
  g.fd_pitch = make_fastdiv(pl.pitch); g.fd_ih1 = make_fastdiv(pl.IH + 1); g.fd_iw1 = make_fastdiv(pl.IW + 1);
  g.nchunk = a.Cs / 32 / pl.splits;
  g.nitems = pl.tiles_m * pl.tiles_n * pl.splits;
  g.c_bytes = (unsigned)c_bytes;
  g.stamps = g_h3_stamps;
  launch_h3_plan(pl, a, g, s);
  return true;
}

}  // namespace dcnn
