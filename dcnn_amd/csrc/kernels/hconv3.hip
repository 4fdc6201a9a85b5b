// Third-generation halo-tiled 3x3 stride-1 convolution (forward and dgrad) for CDNA4.
//
// Why a new kernel (profiles/pmc_conv_r2.md): hconv_kernel runs one 64-deep tap per barrier
// (16 MFMAs per wave between barriers), recomputes every swizzled LDS address per tap (~130
// VALU/SALU instructions per 16 MFMAs) and relies on 2-3 resident workgroups to hide the weight
// ring's latency: 15-21% MFMA busy. This kernel is built around the opposite budget:
//
//  * 8 waves (512 threads), ONE workgroup per CU, each wave owning a 64 (output channels) x 64
//    (pixels) block: 16 accumulator tiles of mfma_f32_16x16x32_bf16.
//  * Roles swapped against hconv_kernel: the weights are the A operand (rows = output
//    channels) and the input halo the B operand (columns = pixels), so an accumulator register
//    quad holds 4 consecutive channels of ONE pixel — the epilogue stores 8 bytes of an NHWC row
//    straight from registers (no LDS staging), and residual / BN masks load the same way.
//  * K step = 32 input channels x one kernel row (3 taps): 48 MFMAs per wave per barrier.
//    The 32-channel halo chunk (64-byte LDS rows) is loaded once per chunk and serves its 3
//    steps; weights stream through a 3-stage ring, two steps ahead, with counted vmcnt waits
//    and raw s_barrier (direct-to-LDS loads stay in flight across barriers).
//  * Every LDS fragment address is precomputed: the A (weight) side is one per-lane base plus
//    immediates; the B (halo) side is 36 per-lane addresses (4 pixel subtiles x 9 taps) plus an
//    immediate buffer offset. The K loop issues 24 ds_read_b128 + 48 MFMA + 3-6 buffer loads
//    and a handful of scalar ops per step.
//  * Bank conflicts: 64-byte rows hold 4 16-byte chunks. A ds_read_b128 is served in four
//    16-lane groups; halo rows read by a group are 16 pixels at an arbitrary tap shift. Pixel
//    subtile row l carries pixel perm(l) (rows 4-11 <- pixels 8-15, rows 12-15 <- pixels 4-7) and
//    the chunk is XOR-swizzled by bit 2 of the halo pixel index: every group then covers 16
//    distinct 16-byte slots for ANY shift (exhaustively checked for 16- and 8-wide tiles); 4-wide
//    tiles use the identity row order and bit 3 (conflict-free at halo pitch 8). Weight rows are
//    16-aligned: swizzle by bit 3 of the row.
//
// Reference parity: the reference runs this GEMM as im2col + cuBLAS SGEMM or cuDNN
// (src/nn/layers_impl/cuda/conv2d_ops.cu:18-128, cudnn_conv2d_ops.cu:187-244).
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "api.h"

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
template <int TWC>
__device__ __forceinline__ int h3_swz(int P) {
  if constexpr (TWC == 4) return ((P >> 3) & 1) << 1;
  return ((P >> 2) & 1) << 1;
}
__device__ __forceinline__ int h3_wswz(int n) { return ((n >> 3) & 1) << 1; }

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void h3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// fixed-order sum over the 16 lanes of a DPP row (rotations by 8 and 4, then quad swaps): every
// lane of the row gets the row total, with no LDS traffic (ds_swizzle / bpermute shuffles cost ~100
// cycles of latency each)
__device__ __forceinline__ float h3_row_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad xor 2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad xor 1
  return v;
}

template <int K, int N, class F>
__device__ __forceinline__ void h3_static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    h3_static_for<K + 1, N>(f);
  }
}

// direct-to-LDS 16-byte load to LDS byte address `base + OFF` (base: one wave-uniform SGPR for the
// whole kernel, OFF an immediate), so the compiler keeps no per-destination M0 constant alive
template <int OFF>
__device__ __forceinline__ void glds16_at(i32x4 rsrc, unsigned base, unsigned voff) {
  asm volatile("s_add_u32 m0, %0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(base), "v"(voff), "s"(rsrc), "n"(OFF)
               : "memory", "m0");
}

// value of lane 0 of this lane's 16-lane DPP row
__device__ __forceinline__ float h3_row_first(float v) {
  // DPP row_newbcast:0 (gfx90a+): lane 0 of each 16-lane row to the whole row, one instruction
  // (four readlanes + selects before)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150, 0xf, 0xf, false));
}

__device__ __forceinline__ bf16x8 lds_b128(const char* smem, int off) {
  return *reinterpret_cast<const bf16x8*>(smem + off);
}
}  // namespace

// geometry the launcher computes once per call
struct H3Geo {
  int TH, TW, IMG, pitch;  // spatial tile IMG x TH x TW pixels; halo row pitch (>= TW + 2)
  int tiles_n, tiles_m;    // channel tiles (N / BN), pixel tiles
  int nchunk;              // 32-channel chunks per split
  int tb[9];               // weight column offset (elements) of tap (dy + 1) * 3 + (dx + 1)
  int halo_bytes;          // bytes of one halo buffer (= 8 waves x HN x 1 KiB)
  int stagger;             // s_sleep(127) count of the second workgroup to arrive on a CU
  unsigned* cu_ctr;        // [2048] per-CU arrival counters + [1] exit ticket (stagger), or null
  int dbg;                 // diagnostic ablations (DCNN_HCONV3_DBG): 1 = no output stores, 2 = no statistics
  unsigned long long* stamps;  // diagnostic: per-wave s_memtime at 8 points (hconv3_set_stamps), or null
};

// NW waves per workgroup (8: one workgroup per CU; 4: two per CU, whose prologue / epilogue
// memory phases overlap each other's MFMA phases), WC of them along the output channels (64
// each), NW / WC along the pixels (64 each). NWS weight stages (3: two steps in flight; 2: one).
// PITCH > 0: compile-time halo row pitch, a multiple of 8 pixels, so a kernel-row (dy) shift keeps
// the bit-2 chunk swizzle and becomes an immediate ds_read offset: 12 halo fragment addresses per
// lane (4 pixel subtiles x 3 dx) instead of 36. PITCH == 0: runtime pitch, 36 addresses.
template <int NW, int WC, int TWC, int HN, int NWI, int NWS, int PITCH>
struct H3 {
  static constexpr int BN = 64 * WC, WP = NW / WC, BM = 64 * WP;
  static constexpr int HALO = NW * HN * 1024;   // one halo buffer
  static constexpr int WST = NW * NWI * 1024;   // one weight stage (3 taps x BN rows x 64 B, padded)
  static constexpr int LDS = 2 * HALO + NWS * WST;
  static_assert(3 * BN * 64 <= WST, "weight stage");
  static_assert(WP * BN * 3 * 4 + 16 <= HALO, "epilogue scratch lives in halo buffer 0");
  static_assert(LDS <= 163840, "LDS budget");
  static_assert(NWS == 2 || NWS == 3, "weight stages");
};

// EPI: epilogue specialisation (compile-time, so the common cases carry no per-option branches
// or selects): 1 = forward with BatchNorm statistics and no bias / residual / ReLU; 2 = data
// gradient with the backward-BatchNorm fusion (optional residual); 0 = any option at run time
template <int NW, int WC, int TWC, int HN, int NWI, int NWS, int PITCH, int EPI = 0>
__global__ void __launch_bounds__(NW * 64, 8 / NW) hconv3_kernel(HConvArgs p, H3Geo g) {
  using T = H3<NW, WC, TWC, HN, NWI, NWS, PITCH>;
  constexpr int BN = T::BN, WP = T::WP;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid % WC, wp = wid / WC;
  const int lr = lane & 15, lh = lane >> 4;
  // diagnostic timeline (off unless hconv3_set_stamps): lane 0 of every wave
  auto stamp = [&](int k) {
    if (g.stamps && lane == 0) g.stamps[((size_t)blockIdx.x * 8 + wid) * 8 + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  // Phase shift of co-resident workgroups: the workgroups of a round run prologue (halo read),
  // K loop and epilogue (output write) in lockstep, so the memory phases are chip-wide bursts
  // during which the MFMAs idle. The second workgroup to arrive on each CU in a launch starts
  // `stagger` x 8K cycles late, so the pair alternates memory and MFMA phases (later rounds
  // inherit the offset: a replacement arrives when its predecessor leaves). Arrival order comes
  // from counters keyed by the hardware CU id (XCC, SE, SH, CU); the grid's last workgroup
  // resets them for the next launch.
  const bool stag = g.stagger > 0 && g.cu_ctr;
  if (stag) {
    volatile int* flag = reinterpret_cast<volatile int*>(smem + T::HALO - 32);
    if (tid == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
      const unsigned key = ((xcc & 7u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
      const unsigned old = __hip_atomic_fetch_add(g.cu_ctr + key, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (int)(old == 1u);
      if (g.stamps) g.stamps[((size_t)blockIdx.x * 8) * 8 + 6] = ((unsigned long long)key << 8) | old;
    }
    __syncthreads();
    const int late = *flag;
    __syncthreads();  // (the flag lives in halo buffer 0, which the prologue overwrites)
    if (late)
      for (int k = 0; k < g.stagger; ++k) __builtin_amdgcn_s_sleep(127);
  }
  const int SPL = p.splits;
  const int u0 = xcd_remap3(blockIdx.x, gridDim.x);
  const int zs = u0 % SPL, lt = u0 / SPL;
  const int tm = lt / g.tiles_n, tn = lt % g.tiles_n;
  const int n0 = tn * BN;
  const int tx_tiles = p.W / g.TW, tpi = tx_tiles * (p.H / g.TH);
  const int ig = tm / tpi, trem = tm - ig * tpi;
  const int y0 = (trem / tx_tiles) * g.TH, x0 = (trem % tx_tiles) * g.TW, img0 = ig * g.IMG;
  const int HW2 = g.TW + 2, HH2 = g.TH + 2, pitch = PITCH > 0 ? PITCH : g.pitch;
  const int HPI = HH2 * pitch;  // halo pixels per image (pitch-padded)
  const int HPX = g.IMG * HPI;  // halo pixels per tile
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += NT) p.zero_ptr[i] = 0.f;
  const i32x4 rsA = raw_rsrc(p.A, p.a_bytes);
  const i32x4 rsB = raw_rsrc(p.B, p.b_bytes);
  const int cbase = zs * g.nchunk * 32;  // first input channel of this split

  // ---- halo loader: instruction k of this wave fills halo pixels [16(wid*HN + k), +16)
  unsigned hsrc[HN];
#pragma unroll
  for (int k = 0; k < HN; ++k) {
    const int P = (wid * HN + k) * 16 + (lane >> 2);
    unsigned v = kOOB3;
    if (P < HPX) {
      const int im = P / HPI, r = P - im * HPI;
      const int hy = r / pitch, hx = r - hy * pitch;
      const int sy = y0 + hy - 1, sx = x0 + hx - 1, n = img0 + im;
      if (hx < HW2 && sy >= 0 && sy < p.H && sx >= 0 && sx < p.W && n < p.NB)
        v = (unsigned)((((long)n * p.H + sy) * p.W + sx) * p.Cs * 2) +
            (unsigned)((cbase + ((lane & 3) ^ h3_swz<TWC>(P)) * 8) * 2);
    }
    hsrc[k] = v;
  }
  // ---- weight loader: stage row R = dx * BN + n (3 taps x BN output channels), 64 B each
  unsigned wsrc[NWI];
  int wtb[NWI][3];  // byte offset of the instruction's tap column for kernel rows dy = 0..2 (SGPRs)
#pragma unroll
  for (int k = 0; k < NWI; ++k) {
    const int R0 = (wid * NWI + k) * 16;  // first stage row of the instruction (wave-uniform)
    const int R = R0 + (lane >> 2);
    const int dx = R0 / BN, n = R - dx * BN;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) wtb[k][dy] = __builtin_amdgcn_readfirstlane(dx < 3 ? g.tb[dy * 3 + dx] * 2 : 0);
    wsrc[k] = (dx < 3 && n0 + n < p.N)
                  ? (unsigned)(((long)(n0 + n) * p.ldb + cbase + ((lane & 3) ^ h3_wswz(n)) * 8) * 2)
                  : kOOB3;
  }
  // LDS byte address of this wave's first halo / weight DMA slot (wave-uniform SGPRs)
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)smem));
  const unsigned hbase = lds0 + wid * HN * 1024, wbase_lds = lds0 + 2 * T::HALO + wid * NWI * 1024;
  auto load_halo = [&](auto buf_c, int c) {
    constexpr int BUF = decltype(buf_c)::value;
    const unsigned co = (unsigned)(c * 64);
    h3_static_for<0, HN>([&](auto kc) {
      constexpr int K = decltype(kc)::value;
      glds16_at<BUF * T::HALO + K * 1024>(rsA, hbase, hsrc[K] + co);
    });
  };
  auto load_w = [&](auto stage_c, int c, int dy) {
    constexpr int ST = decltype(stage_c)::value;
    h3_static_for<0, NWI>([&](auto kc) {
      constexpr int K = decltype(kc)::value;
      glds16_at<ST * T::WST + K * 1024>(rsB, wbase_lds, wsrc[K] + (unsigned)(wtb[K][dy] + c * 64));
    });
  };

  // ---- fragment addresses
  // A (weights): row n = wc*64 + i*16 + lr of stage tap dx: stage + dx*BN*64 + (wc*64 + i*16)*64 + abase
  const int abase = 2 * T::HALO + (wc * 64 + lr) * 64 + ((lh ^ h3_wswz(lr)) << 4);
  // B (halo): pixel subtile j of this wave, tap (dy, dx)
  constexpr int NBA = PITCH > 0 ? 3 : 9;
  static_assert(PITCH == 0 || (PITCH % 8 == 0 && TWC != 4), "dy-invariant swizzle needs pitch % 8 == 0");
  int baddr[4][NBA];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = wp * 64 + j * 16 + h3_perm<TWC>(lr);  // tile-local output pixel
    const int tpx = g.TH * g.TW;
    const int im = q / tpx, r = q - im * tpx;
    const int P0 = im * HPI + (r / g.TW) * pitch + (r % g.TW);  // halo pixel of tap (-1, -1)
#pragma unroll
    for (int t = 0; t < NBA; ++t) {
      const int P = P0 + (NBA == 3 ? t : (t / 3) * pitch + (t % 3));
      baddr[j][t] = P * 64 + ((lh ^ h3_swz<TWC>(P)) << 4);
    }
  }
  auto baddr_of = [&](int j, int dy, int dx) {
    if constexpr (PITCH > 0) return baddr[j][dx] + dy * PITCH * 64;
    else return baddr[j][dy * 3 + dx];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K step: chunk c (halo buffer HB), kernel row DY, weight stage ST. The fragments of tap
  // dx + 1 are read while tap dx's 16 MFMAs run (two register sets in flight), so the LDS latency
  // after the barrier is paid once per step, not once per tap. The step's direct-to-LDS loads
  // (`issue`: next weight stage / next halo, into buffers no wave reads this step) go out after
  // the first MFMAs: an LDS-DMA issue among queued MFMAs costs the wave ~60 cycles instead of
  // delaying the step's first MFMA by its full issue cost (MI355X_MICROARCH cycle constants).
  auto step = [&](auto hb_c, auto dy_c, auto st_c, auto issue) {
    constexpr int HB = decltype(hb_c)::value, DY = decltype(dy_c)::value, ST = decltype(st_c)::value;
    bf16x8 a[3][4], b[3][4];
    auto rd = [&](int dx) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[dx][i] = lds_b128(smem, abase + ST * T::WST + dx * BN * 64 + i * 16 * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[dx][j] = lds_b128(smem, baddr_of(j, DY, dx) + HB * T::HALO);
    };
    auto mm = [&](int dx, int i0, int i1) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = i0; i < i1; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[dx][i], b[dx][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    rd(0);
    rd(1);
    mm(0, 0, 2);
    issue();
    mm(0, 2, 4);
    rd(2);
    mm(1, 0, 4);
    mm(2, 0, 4);
  };
  const int nch = g.nchunk;  // chunks of this split (even, or the single chunk of a 32-channel input)

  if constexpr (NWS == 3) {
    // 3-stage ring, stage = kernel row: step (c, dy) issues the weights of the step two ahead
    // ((c,2) / (c+1,0) / (c+1,1)) and, at dy = 0, the next chunk's halo; the wait after step s
    // retires W(s + 1) and everything older.
    load_halo(I0{}, 0);
    load_w(I0{}, 0, 0);
    load_w(I1{}, 0, 1);
    vmwait<NWI>();
    h3_barrier();
    stamp(1);
    auto chunk = [&](int c, auto hb_c) {
      constexpr int HB = decltype(hb_c)::value;
      const bool more = c + 1 < nch;
      step(hb_c, I0{}, I0{}, [&] {
        load_w(I2{}, c, 2);
        if (more) load_halo(std::integral_constant<int, HB ^ 1>{}, c + 1);
      });
      if (more) vmwait<NWI + HN>(); else vmwait<NWI>();
      h3_barrier();
      step(hb_c, I1{}, I1{}, [&] { if (more) load_w(I0{}, c + 1, 0); });
      if (more) vmwait<NWI>(); else vmwait<0>();
      h3_barrier();
      step(hb_c, I2{}, I2{}, [&] { if (more) load_w(I1{}, c + 1, 1); });
      if (more) vmwait<NWI>(); else vmwait<0>();
      h3_barrier();
    };
    for (int c = 0; c < nch; c += 2) {
      chunk(c, I0{});
      if (c == 0) stamp(2);
      if (c + 1 < nch) chunk(c + 1, I1{});
    }
  } else {
    // 2-stage ring: step s uses stage s & 1 = (c + dy) & 1 and issues W(s + 1) (and, at dy = 0, the
    // next chunk's halo after it); the wait after step s retires W(s + 1) and everything older
    load_halo(I0{}, 0);
    load_w(I0{}, 0, 0);
    vmwait<0>();
    h3_barrier();
    stamp(1);
    auto chunk = [&](int c, auto hb_c) {
      constexpr int HB = decltype(hb_c)::value;
      using S0 = std::integral_constant<int, HB>;
      using S1 = std::integral_constant<int, HB ^ 1>;
      const bool more = c + 1 < nch;
      step(hb_c, I0{}, S0{}, [&] {
        load_w(S1{}, c, 1);
        if (more) load_halo(std::integral_constant<int, HB ^ 1>{}, c + 1);
      });
      if (more) vmwait<HN>(); else vmwait<0>();
      h3_barrier();
      step(hb_c, I1{}, S1{}, [&] { load_w(S0{}, c, 2); });
      vmwait<0>();
      h3_barrier();
      step(hb_c, I2{}, S0{}, [&] { if (more) load_w(S1{}, c + 1, 0); });
      vmwait<0>();
      h3_barrier();
    };
    for (int c = 0; c < nch; c += 2) {
      chunk(c, I0{});
      if (c == 0) stamp(2);
      if (c + 1 < nch) chunk(c + 1, I1{});
    }
  }
  stamp(3);

  // ---------------------------------------------------------------- split-K hand-off
  float* red = reinterpret_cast<float*>(smem);  // epilogue scratch in halo buffer 0 (K loop done)
  if (SPL > 1) {
    // every partial leaves with agent-scope (sc1) 8-byte stores, each wave drains them, one lane
    // adds to the tile's ticket behind the workgroup barrier, and the workgroup whose add returns
    // SPL - 1 reads all partials back with sc1 loads and sums them in split order
    constexpr int E2 = 32;  // float2 pairs per lane
    unsigned long long* part = reinterpret_cast<unsigned long long*>(p.part) + (size_t)lt * SPL * E2 * NT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e2 = (i * 4 + j) * 2 + h;
          const unsigned long long bits = (unsigned long long)__float_as_uint(acc[i][j][2 * h]) |
                                          ((unsigned long long)__float_as_uint(acc[i][j][2 * h + 1]) << 32);
          __hip_atomic_store(part + ((size_t)zs * E2 + e2) * NT + tid, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(smem + T::HALO - 16);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.tickets + lt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(SPL - 1);
      if (last) __hip_atomic_store(p.tickets + lt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    __syncthreads();
    if (!last) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < SPL; ++z) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int e2 = (i * 4 + j) * 2 + h;
            const unsigned long long bits =
                __hip_atomic_load(part + ((size_t)z * E2 + e2) * NT + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc[i][j][2 * h] += __uint_as_float((unsigned)bits);
            acc[i][j][2 * h + 1] += __uint_as_float((unsigned)(bits >> 32));
          }
    }
  }

  // ---------------------------------------------------------------- epilogue (from registers)
  // acc[i][j][r]: channel n0 + wc*64 + i*16 + 4*lh + r, tile pixel wp*64 + j*16 + perm(lr).
  // Every operand load (bias, BN mean / istd, residual, ReLU output, BN input) is issued before the
  // first store: a load's wait also waits for every older store, so interleaving them would make
  // each channel group wait for the previous group's stores to drain.
  bf16* crow[4];                   // output row of pixel subtile j (channel 0)
  const bf16 *rrow[4], *yrow[4], *xrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = wp * 64 + j * 16 + h3_perm<TWC>(lr);
    const int tpx = g.TH * g.TW;
    const int im = q / tpx, r = q - im * tpx;
    const size_t o = (((size_t)(img0 + im) * p.H + y0 + r / g.TW) * p.W + x0 + r % g.TW) * (size_t)p.N;
    crow[j] = p.C + o;
    rrow[j] = p.residual + o;
    yrow[j] = p.bnb.y + o;
    xrow[j] = p.bnb.x + o;
  }
  const bool bnb = EPI == 2 || (EPI == 0 && p.bnb.x != nullptr);
  const bool stats = EPI != 0 || p.stats != nullptr;
  const bool has_res = EPI != 1 && p.residual != nullptr, has_y = bnb && p.bnb.y != nullptr, has_x = bnb && stats;
  const bool has_bias = EPI == 0 && p.bias != nullptr, relu = EPI == 0 && p.relu;
  const int nl = n0 + wc * 64 + 4 * lh;  // this lane's first channel (+ i*16 + r)
  float bv[4][4], mu[4][4], is[4][4];
  uint2 rr[4][4], yy[4][4], xx[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bv[i][r] = has_bias ? p.bias[nl + i * 16 + r] : 0.f;
      mu[i][r] = has_x ? p.bnb.mean[nl + i * 16 + r] : 0.f;
      is[i][r] = has_x ? p.bnb.istd[nl + i * 16 + r] : 0.f;
    }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = nl + i * 16;
      rr[i][j] = has_res ? *reinterpret_cast<const uint2*>(rrow[j] + c) : make_uint2(0u, 0u);
      yy[i][j] = has_y ? *reinterpret_cast<const uint2*>(yrow[j] + c) : make_uint2(0u, 0u);
      xx[i][j] = has_x ? *reinterpret_cast<const uint2*>(xrow[j] + c) : make_uint2(0u, 0u);
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cl0 = wc * 64 + i * 16 + 4 * lh;  // tile-local first of this lane's 4 channels
    float gv[4][4], xh[4][4];  // [j][r]: stored value, and (bnb) stored value * xhat
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float f[4];
      const bf16* rb = reinterpret_cast<const bf16*>(&rr[i][j]);
      const bf16* yb = reinterpret_cast<const bf16*>(&yy[i][j]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f[r] = acc[i][j][r] + bv[i][r];
        if (has_res) f[r] += (float)rb[r];
        if (relu) f[r] = fmaxf(f[r], 0.f);
        if (has_y) f[r] = (float)yb[r] > 0.f ? f[r] : 0.f;
      }
      uint2 o;
      bf16* ob = reinterpret_cast<bf16*>(&o);
#pragma unroll
      for (int r = 0; r < 4; ++r) ob[r] = (bf16)f[r];
      if (!(g.dbg & 1)) *reinterpret_cast<uint2*>(crow[j] + nl + i * 16) = o;
      const bf16* xb = reinterpret_cast<const bf16*>(&xx[i][j]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gv[j][r] = (float)ob[r];  // statistics of the values actually stored
        xh[j][r] = gv[j][r] * (((float)xb[r] - mu[i][r]) * is[i][r]);
      }
    }
    if (stats && !(g.dbg & 2)) {
      float pv[4], sa[4], sb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (bnb) {
          pv[r] = 0.f;
          sa[r] = (gv[0][r] + gv[1][r]) + (gv[2][r] + gv[3][r]);
          sb[r] = (xh[0][r] + xh[1][r]) + (xh[2][r] + xh[3][r]);
        } else {
          // forward Welford rows: sums about a pivot (the wave's first pixel of the channel: lane
          // 16*lh of the DPP row, broadcast by a row rotation chain-free read)
          pv[r] = h3_row_first(gv[0][r]);
          float a = 0.f, b = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) { const float d = gv[j][r] - pv[r]; a += d; b += d * d; }
          sa[r] = a;
          sb[r] = b;
        }
        sa[r] = h3_row_sum(sa[r]);  // fixed-order sum over the 16 lanes (pixels) of the DPP row
        sb[r] = h3_row_sum(sb[r]);
      }
      if (lr == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* e = red + (wp * BN + cl0 + r) * 3;
          e[0] = pv[r];
          e[1] = sa[r];
          e[2] = sb[r];
        }
      }
    }
  }
  stamp(4);
  if (stats) {
    __syncthreads();
    if (tid < BN) {
      if (bnb) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < WP; ++w) { a += red[(w * BN + tid) * 3 + 1]; b += red[(w * BN + tid) * 3 + 2]; }
        p.stats[((long)tm * 2 + 0) * p.N + n0 + tid] = a;
        p.stats[((long)tm * 2 + 1) * p.N + n0 + tid] = b;
      } else {
        Welford w = welford_from_shifted(64.f, red[tid * 3 + 0], red[tid * 3 + 1], red[tid * 3 + 2]);
#pragma unroll
        for (int k = 1; k < WP; ++k) {
          const float* e = red + (k * BN + tid) * 3;
          w = welford_merge(w, welford_from_shifted(64.f, e[0], e[1], e[2]));
        }
        store_welford(p.stats, tm, p.N, n0 + tid, w);
      }
    }
  }
  stamp(5);
  if (stag) {
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(smem + T::HALO - 32);
    if (tid == 0) {
      const unsigned done = __hip_atomic_fetch_add(g.cu_ctr + 2048, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (int)(done == gridDim.x - 1);
    }
    __syncthreads();
    if (*flag) {  // every workgroup has arrived: counters back to zero for the next launch
      for (int i = tid; i <= 2048; i += NT) __hip_atomic_store(g.cu_ctr + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
int hconv_split_target();  // hconv.hip (DCNN_HCONV_SPLIT / hconv_set_split_target; 0 = never split)

static int g_h3 = [] {
  const char* e = getenv("DCNN_HCONV3");
  return e ? atoi(e) : 1;
}();
void hconv3_enable(int on) { g_h3 = on; }
static unsigned long long* g_h3_stamps = nullptr;
static int g_h3_dbg = [] {
  const char* e = getenv("DCNN_HCONV3_DBG");
  return e ? atoi(e) : 0;
}();
static int g_h3_stagger = [] {
  const char* e = getenv("DCNN_HCONV3_STAGGER");
  return e ? atoi(e) : 0;
}();
void hconv3_set_stagger(int sleeps) { g_h3_stagger = sleeps; }
void hconv3_set_stamps(uintptr_t p) { g_h3_stamps = reinterpret_cast<unsigned long long*>(p); }

struct H3Plan {
  int WC, TWC, HN, NWI, TH, TW, IMG, pitch, splits, tiles_m, tiles_n;
};

// tile plan for a 3x3 stride-1 conv of NB x H x W pixels, Cs input / N output channels
bool hconv3_plan(int NB, int H, int W, int Cs, int N, int ntaps, H3Plan* pl) {
  // an even 32-channel chunk count (split-K pairs), or one chunk (32 input channels: ResNet-18's
  // first residual conv)
  if (!g_h3 || ntaps != 9 || (Cs % 64 && Cs != 32) || N % 64) return false;
  // 16-wide (and wider) maps: 4-wave workgroups of 64 channels x one 16x16 tile, two per CU
  // (LDS 72 KB). The 8- and 4-wide maps stay on hconv_kernel (measured faster there: their split-K
  // grids of single 8-wave workgroups lose more to the serial prologue / epilogue than the K loop
  // gains).
  // 8x8 maps (DCNN_HCONV3_8=1, experiment): 4 images of 8x8 per 256-pixel tile, halo pitch 10
  static const int on8 = [] { const char* e = getenv("DCNN_HCONV3_8"); return e ? atoi(e) : 0; }();
  const bool m8 = on8 && W == 8 && H == 8 && NB % 4 == 0;
  if (!m8 && (W % 16 || H % 16)) return false;
  const int WC = 1, NW = 4, BN = 64, BM = 256;
  const int TW = m8 ? 8 : 16, TWC = TW, TH = m8 ? 8 : 16, IMG = m8 ? 4 : 1;
  const int NWI = (3 * BN / 16 + NW - 1) / NW;
  const int pitch = TW + 2;
  const int HN = (IMG * (TH + 2) * pitch + 16 * NW - 1) / (16 * NW);
  // the instances: <4, 1, 16, 6, 3, 2, 0> (16-wide maps), <4, 1, 8, 7, 3, 2, 0> (8x8 maps)
  if (!((TWC == 16 && HN == 6) || (TWC == 8 && HN == 7)) || NWI != 3) return false;
  pl->WC = WC; pl->TWC = TWC; pl->HN = HN; pl->NWI = NWI;
  pl->TH = TH; pl->TW = TW; pl->IMG = IMG; pl->pitch = pitch;
  pl->tiles_m = NB * H * W / BM;
  pl->tiles_n = N / BN;
  // split-K over 32-channel chunks until the grid holds the target workgroup count (two resident
  // per CU), keeping an even chunk count per split
  const long tiles = (long)pl->tiles_m * pl->tiles_n;
  const int nchunk = Cs / 32, target = hconv_split_target();
  int s = 1;
  while (tiles * s < target && nchunk % (4 * s) == 0) s *= 2;
  pl->splits = s;
  return true;
}

template <int NW, int WC, int TWC, int HN, int NWI, int NWS, int PITCH, int EPI>
static void launch_h3e(const HConvArgs& a, const H3Geo& g, int grid, hipStream_t s) {
  using T = H3<NW, WC, TWC, HN, NWI, NWS, PITCH>;
  auto k = hconv3_kernel<NW, WC, TWC, HN, NWI, NWS, PITCH, EPI>;
  static bool attr = false;
  if (!attr) {
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS));
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), T::LDS, s, a, g);
  DCNN_LAUNCH_CHECK();
}

static int g_h3_epi = [] {  // DCNN_HCONV3_EPI=0: always the generic epilogue (A/B)
  const char* e = getenv("DCNN_HCONV3_EPI");
  return e ? atoi(e) : 1;
}();

template <int NW, int WC, int TWC, int HN, int NWI, int NWS, int PITCH>
static void launch_h3(const HConvArgs& a, const H3Geo& g, int grid, hipStream_t s) {
  const bool plain_fwd = a.stats && !a.bnb.x && !a.residual && !a.relu && !a.bias;
  const bool bnb_dgrad = a.stats && a.bnb.x && !a.relu && !a.bias;
  if (g_h3_epi && plain_fwd) return launch_h3e<NW, WC, TWC, HN, NWI, NWS, PITCH, 1>(a, g, grid, s);
  if (g_h3_epi && bnb_dgrad) return launch_h3e<NW, WC, TWC, HN, NWI, NWS, PITCH, 2>(a, g, grid, s);
  launch_h3e<NW, WC, TWC, HN, NWI, NWS, PITCH, 0>(a, g, grid, s);
}

static void launch_h3_plan(const H3Plan& pl, const HConvArgs& a, const H3Geo& g, int grid, hipStream_t s) {
  if (pl.WC == 1 && pl.TWC == 16 && pl.HN == 6 && pl.NWI == 3) return launch_h3<4, 1, 16, 6, 3, 2, 0>(a, g, grid, s);
  if (pl.WC == 1 && pl.TWC == 8 && pl.HN == 7 && pl.NWI == 3) return launch_h3<4, 1, 8, 7, 3, 2, 0>(a, g, grid, s);
  throw std::runtime_error("hconv3: no kernel instance for this plan");
}

// returns false when the shape / taps / epilogue options are not covered (caller falls back)
bool hconv3_try(const HConvArgs& a0, hipStream_t s) {
  H3Plan pl;
  if (a0.Cf || a0.fold.part || !hconv3_plan(a0.NB, a0.H, a0.W, a0.Cs, a0.N, a0.ntaps, &pl)) return false;
  H3Geo g{};
  for (int t = 0; t < 9; ++t) g.tb[t] = -1;
  for (int t = 0; t < a0.ntaps; ++t) {
    const int dy = a0.tap_dy[t], dx = a0.tap_dx[t];
    if (dy < -1 || dy > 1 || dx < -1 || dx > 1) return false;
    g.tb[(dy + 1) * 3 + dx + 1] = a0.tap_b[t];
  }
  for (int t = 0; t < 9; ++t)
    if (g.tb[t] < 0) return false;
  if (a0.a_bytes >= 0x80000000u || a0.b_bytes >= 0x80000000u) return false;
  HConvArgs a = a0;
  if (a.splits != pl.splits) throw std::runtime_error("hconv3: split count mismatch (use hconv_splits)");
  if (pl.splits > 1 && (!a.part || !a.tickets)) throw std::runtime_error("hconv3: split-K workspace missing");
  g.TH = pl.TH; g.TW = pl.TW; g.IMG = pl.IMG; g.pitch = pl.pitch;
  g.tiles_n = pl.tiles_n; g.tiles_m = pl.tiles_m;
  g.nchunk = a.Cs / 32 / pl.splits;
  g.halo_bytes = 4 * pl.HN * 1024;
  g.stamps = g_h3_stamps;
  g.dbg = g_h3_dbg;
  const int grid = pl.tiles_m * pl.tiles_n * pl.splits;
  static unsigned* ctr = nullptr;
  if (pl.splits == 1 && g_h3_stagger > 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DCNN_HIP_CHECK(hipStreamIsCapturing(s, &cs));
    if (!ctr && cs == hipStreamCaptureStatusNone) {  // (never allocated inside a capture)
      DCNN_HIP_CHECK(hipMalloc(&ctr, 2049 * sizeof(unsigned)));
      DCNN_HIP_CHECK(hipMemset(ctr, 0, 2049 * sizeof(unsigned)));
      DCNN_HIP_CHECK(hipDeviceSynchronize());
    }
    g.cu_ctr = ctr;
    g.stagger = ctr ? g_h3_stagger : 0;
  }
  launch_h3_plan(pl, a, g, grid, s);
  return true;
}

}  // namespace dcnn
