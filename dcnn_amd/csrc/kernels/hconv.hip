// Halo-tiled direct convolution for stride-1 convolutions with a 1-pixel reach (3x3 pad 1,
// and the dgrad of such a conv) on CDNA4 MFMA 16x16x32 bf16.
//
// The gathered implicit GEMM (gemm2.hip) re-fetches every input pixel once per kernel tap
// (9x for 3x3) through L2, which bounds the N=64..128 layers at ~40-60 flop/byte. Here a
// workgroup owns a spatial output tile (IMG images x TH x TW pixels = BM GEMM rows) and stages
// the *halo* of that tile — (TH+2) x (TW+2) pixels x 64 input channels — into LDS once per
// channel chunk with 16-byte direct-to-LDS loads (out-of-image halo pixels zero-filled by the
// buffer range check). All taps then read their A fragments from the same halo image at a
// per-tap row offset, so the input is read ~1.3-2.3x instead of 9x; only the (small, L2
// resident) weight slice is streamed per tap.
//
//   K loop: for each 64-channel chunk c: halo(c) [prefetched one chunk ahead]
//             for each tap t: B(c, t) [ring of NBS LDS stages, NBS - 1 steps ahead, counted
//                                      vmcnt waits], MFMA over 64 channels
//
// A step is only TM x TN x 2 MFMAs per wave (8 for the 64x64 tiles of the 4x4 layers), far
// shorter than an L2 round trip, so a one-step-ahead weight prefetch leaves the loop latency
// bound; the deeper ring keeps two steps in flight.
//
// The epilogue is the gemm2 one (bias, residual, ReLU, BatchNorm partial statistics, 16-byte
// stores through an LDS-staged bf16 tile), with the spatial-tile -> NHWC row mapping.
#include <cstdio>

#include "common.h"
#include "api.h"
#include "hconv3_plan.h"

namespace dcnn {


namespace {
constexpr unsigned kOOBh = 0x80000000u;

// opaque to the compiler's wait-count pass: the manual vmcnt waits of the B ring below are the
// only synchronisation of these LDS writes (a visible LDS DMA would be drained before every
// ds_read, defeating the ring)
__device__ __forceinline__ void glds16h(i32x4 rsrc, char* lds, unsigned voff) { glds16_opaque(rsrc, lds, voff); }

// wait until at most m * U of this lane's direct-to-LDS loads are outstanding (m in 0..2)
template <int U>
__device__ __forceinline__ void vm_wait_groups(int m) {
  if (m <= 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (m == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * U) : "memory");
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int xcd_remap_h(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// 128-byte LDS rows (64 bf16 channels), 16-byte chunks XOR-swizzled by the row's low 3 bits
__device__ __forceinline__ int hoff(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

// Output pixel of A-fragment row l (0..15) of a 16-row subtile. ds_read_b128 serves a wave in
// four 16-lane groups ({0-3,12-15,20-27}, ...; MI355X_MICROARCH LDS table) over 64 banks =
// 256 B, i.e. (row parity, swizzled chunk) must differ across a group. With 16-wide tiles a
// subtile is 16 consecutive halo rows and the identity is conflict-free; on 8-wide tiles
// (halo pitch 10) lanes 0-3 and 12-15 landed on halo rows 16 apart (same bank set: 2-way
// conflicts, ~2.5 extra LDS cycles per read measured on the 8x8 layer) and likewise on 4-wide
// tiles (pitch 6). Permuting which pixel each fragment row carries makes every group hit 8
// distinct (parity, chunk) slots per 8 lanes; the epilogue stages row l's results at pixel
// hperm(l), so outputs are unchanged (and bit-identical: each element's K order is the same).
__device__ __forceinline__ int hperm(int l, int tw) {
  if (tw == 8) return l < 4 ? l : (l < 12 ? l + 4 : l - 8);   // rows 4-11 <- pixels 8-15
  if (tw == 4) return l < 8 ? l : (l < 12 ? l + 4 : l - 4);   // rows 8-11 <- pixels 12-15
  return l;
}
}  // namespace

// TPS taps per K step (one barrier per step), NHB halo buffers (1 when there is a single
// 64-channel chunk: nothing to prefetch), NBS weight stages (NBS - 1 steps in flight)
template <int BM, int BN, int TPS, int NHB, int NBS, bool F32O = false>
struct HC {
  // wave layout: 2 x 2 waves, or 4 x 1 (all four waves along M) for tall 256 x 64 tiles, where
  // each wave then owns a 64 x 64 block (twice the MFMAs per LDS fragment read of a 2 x 2 split)
  static constexpr int WN = (BM >= 4 * BN) ? 1 : 2, WM = 4 / WN;
  static constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 16x16 subtiles per wave
  static constexpr int BTAP = BN * 128;                  // bytes of one tap's weight slice
  static constexpr int BST = TPS * BTAP;                 // bytes per weight stage
  static constexpr int B_INS = BN / 32;                  // glds per wave per tap slice
  static constexpr int OB = F32O ? 4 : 2;                // bytes per staged output element
  static constexpr int EPI_PITCH = BN * OB + 16;
  // dynamic LDS: NHB halo buffers of HALO = 128 * (halo rows padded to 32) bytes, then NBS weight stages
  static int lds_bytes(int halo) {
    const int main = NHB * halo + NBS * BST, epi = BM * EPI_PITCH;
    return main > epi ? main : epi;
  }
};

// Shared epilogue of the halo convs: acc (+bias) -> bf16 (F32O: fp32) tile staged in LDS `smem`
// (>= BM x EPI_PITCH bytes) -> NHWC rows (+residual, ReLU, backward-BN mask) and the tile's
// BatchNorm statistics row `tm`. Contains block barriers: every thread of the workgroup must call it.
template <bool F32O>
__device__ __forceinline__ void load_row8(const char* src, float* f) {
  if (F32O) {
    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 16);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    unpack8(*reinterpret_cast<const uint4*>(src), f);
  }
}

template <int BM, int BN, bool F32O>
__device__ __forceinline__ void hc_epilogue(const HConvArgs& p,
                                            f32x4 (&acc)[HC<BM, BN, 1, 1, 2, F32O>::TM][HC<BM, BN, 1, 1, 2, F32O>::TN],
                                            char* smem, int n0,
                                            int tm, int img0, int y0, int x0) {
  using T = HC<BM, BN, 1, 1, 2, F32O>;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / T::WN, wn = wid % T::WN;
  // ---- epilogue 1: acc (+bias) -> bf16 LDS tile [BM][BN] ----
#pragma unroll
  for (int j = 0; j < T::TN; ++j) {
    const int col = wn * (BN / T::WN) + j * 16 + (lane & 15);
    const float bv = (p.bias && n0 + col < p.N) ? p.bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / T::WM) + i * 16 + hperm((lane >> 4) * 4 + r, p.TW);
        if (F32O)
          *reinterpret_cast<float*>(smem + row * T::EPI_PITCH + col * 4) = acc[i][j][r] + bv;
        else
          *reinterpret_cast<bf16*>(smem + row * T::EPI_PITCH + col * 2) = (bf16)(acc[i][j][r] + bv);
      }
  }
  __syncthreads();
  // ---- epilogue 2: 16-byte rows -> NHWC global (+residual, ReLU, BN partial stats) ----
  constexpr int CG = BN / 8;
  constexpr int RSTEP = 256 / CG;
  const int cg = tid % CG, r0 = tid / CG;
  const int ncol = n0 + cg * 8;
  const bool cok = ncol < p.N;  // (N = 32: the upper half of the 64-column tile is padding)
  float s[8], q[8], mu[8], is[8], pv[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) s[v] = q[v] = mu[v] = is[v] = pv[v] = 0.f;
  const bool bnb = !F32O && p.bnb.x != nullptr;  // backward-BN fusion (api.h BnbArgs; bf16 output only)
  if (bnb && cok) {
#pragma unroll
    for (int v = 0; v < 8; ++v) { mu[v] = p.bnb.mean[ncol + v]; is[v] = p.bnb.istd[ncol + v]; }
  }
  // forward statistics are summed about a pivot (tile row 0 of the column, a value of the tile
  // itself) and leave as a (count, mean, M2) triple: no E[x^2] - mean^2 cancellation
  float piv_col = 0.f;
  if (p.stats && !bnb) {
    load_row8<F32O>(smem + cg * 8 * T::OB, pv);
    if (tid < BN)
      piv_col = F32O ? *reinterpret_cast<const float*>(smem + tid * 4) : (float)*reinterpret_cast<const bf16*>(smem + tid * 2);
  }
  const int tpx = p.TH * p.TW;
  for (int row = r0; row < BM; row += RSTEP) {
    const int im = row / tpx, r2 = row - im * tpx;
    const int n = img0 + im;
    if (n >= p.NB || !cok) continue;
    const long orow = ((long)n * p.H + y0 + r2 / p.TW) * p.W + x0 + r2 % p.TW;
    float f[8];
    load_row8<F32O>(smem + row * T::EPI_PITCH + cg * 8 * T::OB, f);
    if (F32O ? p.residual_f != nullptr : p.residual != nullptr) {
      float rr[8];
      if (F32O)
        load_row8<true>(reinterpret_cast<const char*>(p.residual_f + orow * p.N + ncol), rr);
      else
        unpack8(*reinterpret_cast<const uint4*>(p.residual + orow * p.N + ncol), rr);
#pragma unroll
      for (int v = 0; v < 8; ++v) f[v] += rr[v];
    }
    if (p.relu) {
#pragma unroll
      for (int v = 0; v < 8; ++v) f[v] = fmaxf(f[v], 0.f);
    }
    if (bnb && p.bnb.y) {
      float yo[8];
      unpack8(*reinterpret_cast<const uint4*>(p.bnb.y + orow * p.N + ncol), yo);
#pragma unroll
      for (int v = 0; v < 8; ++v) f[v] = yo[v] > 0.f ? f[v] : 0.f;
    }
    float g[8];
    if (F32O) {
      float* dst = p.Cf + orow * p.N + ncol;
      *reinterpret_cast<float4*>(dst) = make_float4(f[0], f[1], f[2], f[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(f[4], f[5], f[6], f[7]);
#pragma unroll
      for (int v = 0; v < 8; ++v) g[v] = f[v];
    } else {
      const uint4 o = pack8(f);
      *reinterpret_cast<uint4*>(p.C + orow * p.N + ncol) = o;
      unpack8(o, g);  // statistics of the values actually stored
    }
    if (p.stats) {
      if (bnb) {
        float xv[8];
        unpack8(*reinterpret_cast<const uint4*>(p.bnb.x + orow * p.N + ncol), xv);
#pragma unroll
        for (int v = 0; v < 8; ++v) { s[v] += g[v]; q[v] += g[v] * (xv[v] - mu[v]) * is[v]; }
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v) { const float d = g[v] - pv[v]; s[v] += d; q[v] += d * d; }
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
      for (int cc = tid; cc < 2 * BN; cc += 256) {
        const int which = cc / BN, c2 = cc % BN;
        if (n0 + c2 >= p.N) continue;
        float a = 0.f;
        for (int k = 0; k < RSTEP; ++k) a += red[(k * 2 + which) * BN + c2];
        *&p.stats[((long)tm * 2 + which) * p.N + n0 + c2] = a;
      }
    } else if (tid < BN && n0 + tid < p.N) {  // forward: Welford triple [tiles][3][N], fixed summation order
      float a = 0.f, b = 0.f;
      for (int k = 0; k < RSTEP; ++k) { a += red[(k * 2 + 0) * BN + tid]; b += red[(k * 2 + 1) * BN + tid]; }
      const float cnt = (float)(min(p.IMG, p.NB - img0) * tpx);
      const Welford w = welford_from_shifted(cnt, piv_col, a, b);
      store_welford(p.stats, tm, p.N, n0 + tid, w);
    }
  }
}

template <int BM, int BN, int TPS, int NHB, int NBS, bool F32O>
__global__ void __launch_bounds__(256, 1) hconv_kernel(HConvArgs p) {
  prefetch_kernargs<sizeof(HConvArgs)>();
  using T = HC<BM, BN, TPS, NHB, NBS, F32O>;
  static_assert(NBS >= 2 && NBS <= 4 && (NBS == 2 || TPS == 1), "deep weight ring needs 1 tap per step");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  struct { int HALO; } T_rt{p.HPR * 128};
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / T::WN, wn = wid % T::WN;
  const int tiles_n = (p.N + BN - 1) / BN;  // (N = 32: one half-filled column tile)
  const int SPL = p.splits;                      // workgroups per output tile (split-K)
  const int lt0 = xcd_remap_h(blockIdx.x, gridDim.x);
  const int zs = lt0 % SPL, lt = lt0 / SPL;      // this workgroup's split, output tile
  const int tm = lt / tiles_n, tn = lt % tiles_n;
  const int n0 = tn * BN;
  // spatial tile tm -> (image group, tile row, tile col)
  const int tx_tiles = p.W / p.TW, ty_tiles = p.H / p.TH;
  const int tpi = tx_tiles * ty_tiles;
  const int ig = tm / tpi, trem = tm - ig * tpi;
  const int y0 = (trem / tx_tiles) * p.TH, x0 = (trem % tx_tiles) * p.TW;
  const int img0 = ig * p.IMG;
  const int HW2 = p.TW + 2, HH2 = p.TH + 2, HPI = HH2 * HW2;  // halo pixels per image
  const int HP = p.IMG * HPI;
  if (p.zero_ptr && blockIdx.x == 0)
    for (int i = tid; i < p.zero_n; i += 256) p.zero_ptr[i] = 0.f;

  const i32x4 rsA = raw_rsrc(p.A, p.a_bytes);
  const i32x4 rsB = raw_rsrc(p.B, p.b_bytes);

  // ---- halo loader: per-lane pixel base offsets for its rows (fixed across chunks) ----
  const int hch = lane & 7;                               // physical chunk slot
  const int HNI = (HP + 31) / 32;                         // glds per wave per halo chunk (8 rows each)
  constexpr int HMAX = BM >= 256 ? 12 : 10;  // halo loads per lane (the wide tiles' 18x18 halo: 11)
  unsigned h_base[HMAX];
  int h_row[HMAX];
#pragma unroll
  for (int j = 0; j < HMAX; ++j) {
    h_base[j] = kOOBh;
    h_row[j] = 0;
    if (j < HNI) {
      const int row = (wid * HNI + j) * 8 + (lane >> 3);
      h_row[j] = row;
      if (row < HP) {
        const int im = row / HPI, r2 = row - im * HPI;
        const int sy = y0 + r2 / HW2 - 1, sx = x0 + r2 % HW2 - 1;
        const int n = img0 + im;
        if (sy >= 0 && sy < p.H && sx >= 0 && sx < p.W && n < p.NB)
          h_base[j] = (unsigned)((((long)n * p.H + sy) * p.W + sx) * p.Cs * 2);
      }
    }
  }
  auto load_halo = [&](int buf, int c0) {
    char* Hs = smem + buf * T_rt.HALO;
#pragma unroll
    for (int j = 0; j < HMAX; ++j) {
      if (j < HNI) {
        const int lch = hch ^ (h_row[j] & 7);
        const unsigned voff = h_base[j] == kOOBh ? kOOBh : h_base[j] + (unsigned)((c0 + lch * 8) * 2);
        glds16h(rsA, Hs + (wid * HNI + j) * 1024, voff);
      }
    }
  };
  // ---- weight loader: B[n0 + row][tap_b[t] + c0 + chunk*8] ----
  unsigned b_base[T::B_INS];
  int b_lch[T::B_INS];
#pragma unroll
  for (int i = 0; i < T::B_INS; ++i) {
    const int row = (wid * T::B_INS + i) * 8 + (lane >> 3);
    b_lch[i] = hch ^ (row & 7);
    b_base[i] = (unsigned)((long)(n0 + row) * p.ldb * 2);
  }
  auto load_b = [&](int buf, int c0, int t0) {
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int t = t0 + u;
      if (TPS > 1 && t >= p.ntaps) break;
      char* Bs = smem + NHB * T_rt.HALO + buf * T::BST + u * T::BTAP;
#pragma unroll
      for (int i = 0; i < T::B_INS; ++i)
        glds16h(rsB, Bs + (wid * T::B_INS + i) * 1024, b_base[i] + (unsigned)((p.tap_b[t] + c0 + b_lch[i] * 8) * 2));
    }
  };

  // ---- per-lane A rows: halo row of tap (0, 0) for each M subtile ----
  int arow0[T::TM];
#pragma unroll
  for (int i = 0; i < T::TM; ++i) {
    const int m = wm * (BM / T::WM) + i * 16 + hperm(lane & 15, p.TW);   // tile-local output row
    const int tpx = p.TH * p.TW;
    const int im = m / tpx, r2 = m - im * tpx;
    arow0[i] = im * HPI + (r2 / p.TW + 1) * HW2 + (r2 % p.TW + 1);
  }

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunk = p.Cs / 64 / SPL;          // channel chunks of this split
  const int cbase = zs * nchunk * 64;          // its first channel
  const int spc = (p.ntaps + TPS - 1) / TPS;  // K steps per channel chunk
  const int nsteps = nchunk * spc;
  // step j's weights live in stage j % NBS; step k + NBS - 1 is issued at the top of step k into
  // the stage step k - 1 consumed. The halo of chunk c + 1 is issued at the first step of chunk
  // c ahead of that step's weights, so it is always older than the weight stages a wait leaves
  // in flight and the per-step wait counts only weight loads.
  constexpr int BU = TPS * T::B_INS;  // weight loads per lane per step
  auto step_ct = [&](int j, int* cj, int* tj) { *cj = j / spc; *tj = (j - *cj * spc) * TPS; };
  load_halo(0, cbase);
#pragma unroll
  for (int j = 0; j < NBS - 1; ++j) {
    if (j < nsteps) {
      int cj, tj;
      step_ct(j, &cj, &tj);
      load_b(j, cbase + cj * 64, tj);
    }
  }
  vm_wait_groups<BU>(min(NBS - 2, nsteps - 1));
  lds_barrier();
  int bcur = 0;
  for (int k = 0; k < nsteps; ++k) {
    const int c = k / spc, t0 = (k - c * spc) * TPS;
    // the next chunk's halo goes out BEFORE this step's weight stage: the end-of-step wait leaves
    // only the newest (NBS - 2) weight stages in flight, so the halo has landed by the next step
    // whatever the steps per chunk
    if (NHB == 2 && t0 == 0 && c + 1 < nchunk) load_halo((c + 1) & 1, cbase + (c + 1) * 64);
    if (k + NBS - 1 < nsteps) {
      int cj, tj;
      step_ct(k + NBS - 1, &cj, &tj);
      load_b(bcur == 0 ? NBS - 1 : bcur - 1, cbase + cj * 64, tj);
    }
    const char* Hs = smem + (NHB == 2 ? (c & 1) : 0) * T_rt.HALO;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int t = t0 + u;
      if (TPS > 1 && t >= p.ntaps) break;
      const char* Bs = smem + NHB * T_rt.HALO + bcur * T::BST + u * T::BTAP;
      const int toff = p.tap_dy[t] * HW2 + p.tap_dx[t];
      // both k-halves' fragments are read up front: the second half's LDS latency hides behind
      // the first half's MFMAs instead of sitting between them
      bf16x8 a[2][T::TM], b[2][T::TN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < T::TM; ++i) a[kk][i] = *reinterpret_cast<const bf16x8*>(Hs + hoff(arow0[i] + toff, ch));
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          b[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + hoff(wn * (BN / T::WN) + j * 16 + (lane & 15), ch));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < T::TM; ++i)
#pragma unroll
          for (int j = 0; j < T::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    // step k + 1's weights (and halo) landed for this lane, then for the whole workgroup
    vm_wait_groups<BU>(min(NBS - 2, nsteps - 2 - k));
    lds_barrier();
    bcur = bcur == NBS - 1 ? 0 : bcur + 1;
  }

  if constexpr (T::WN == 2) if (SPL > 1) {  // (the 4 x 1 wide tiles never split: host)
    // split-K hand-off without fences (MI355X_MICROARCH "Valid forms" row 1): every partial is
    // stored with agent-scope (sc1) 16-byte buffer stores ([split][tile i, j][lane]), each wave
    // drains them, one lane adds to the tile's ticket after the workgroup barrier, and the
    // workgroup whose add returns SPL - 1 reads the partials back with sc1 loads (all of a split
    // in flight at once) and sums them in split order.
    constexpr int NE = T::TM * T::TN;  // 16-byte accumulator tiles per lane
    const __amdgpu_buffer_rsrc_t rsP =
        __builtin_amdgcn_make_buffer_rsrc(p.part + (size_t)lt * SPL * NE * 256 * 4, 0, SPL * NE * 256 * 16, 0x00020000);
    constexpr int kSC1 = 16;  // cache policy: sc1 (agent-coherent)
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsP,
                                               ((zs * NE + i * T::TN + j) * 256 + tid) * 16, 0, kSC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(smem);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(p.tickets + lt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(SPL - 1);
      if (last) __hip_atomic_store(p.tickets + lt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    const int last = *flag;
    __syncthreads();  // the epilogue reuses smem
    if (!last) return;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < SPL; ++z) {
      f32x4 t[NE];
#pragma unroll
      for (int k = 0; k < NE; ++k)
        t[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsP, ((z * NE + k) * 256 + tid) * 16, 0, kSC1));
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j) acc[i][j] += t[i * T::TN + j];
    }
  }

  hc_epilogue<BM, BN, F32O>(p, acc, smem, n0, tm, img0, y0, x0);
}


// ---------------------------------------------------------------------------------------------
// host side: tile geometry + dispatch
// ---------------------------------------------------------------------------------------------
// Output tile = IMG images x TH x TW pixels = BM rows; needs W % TW == 0, H % TH == 0.
static bool hconv_geometry(int NB, int H, int W, int BM, int* TH, int* TW, int* IMG) {
  int tw = W >= 16 ? 16 : W;
  if (W % tw) return false;
  int th = BM / tw;
  if (th > H) th = H;
  if (th <= 0 || H % th || BM % (th * tw)) return false;
  const int img = BM / (th * tw);
  if ((img * (th + 2) * (tw + 2)) > 384) return false;  // halo loader: <= 12 x 32 rows
  *TH = th; *TW = tw; *IMG = img;
  (void)NB;
  return true;
}

static void hconv_pick(const HConvArgs& a, int* bm, int* bn) {
  // prefer 128 x 128 when it still gives >= ~1.5 workgroups per CU, else shrink
  auto tiles = [&](int m, int n) { return (long)((a.NB * a.H * a.W + m - 1) / m) * ((a.N + n - 1) / n); };
  *bm = 128;
  *bn = (a.N % 128 == 0 && tiles(128, 128) >= 384) ? 128 : 64;
  if (tiles(*bm, *bn) < 384) {
    // small maps (4x4 layer-4 convs at batch 256): 64 x 128 tiles (twice the MFMAs per K step,
    // split-K refills the grid) while they still give one tile per CU; 64 x 64 below that.
    // Measured: 4x4x512 forward 46.5 -> 40.9 us, dgrad 44.8 -> 39.5 us (tools/gpu_convsplit.sh tile)
    *bm = 64;
    *bn = (a.N % 128 == 0 && tiles(64, 128) >= 256) ? 128 : 64;
  }
}

bool hconv_supported(int NB, int H, int W, int Cs, int N, int ntaps) {
  // N = 32 runs as a 64-column tile whose upper half reads zero weights (buffer range check) and
  // is never stored: the 32-channel data gradient of a 32 -> 64 channel conv (ResNet-18 layer 1)
  // Cs = 32 (one 32-channel chunk) only on the hconv3 kernel
  if (Cs == 32) {
    H3Plan pl;
    return hconv3_plan(NB, H, W, Cs, N, ntaps, &pl);
  }
  if (Cs % 64 || (N % 64 && N != 32) || ntaps < 1 || ntaps > 9) return false;
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn, th, tw, img;
  hconv_pick(a, &bm, &bn);
  if (!hconv_geometry(NB, H, W, bm, &th, &tw, &img)) return false;
  return NB % img == 0;
}

// target workgroup count of the split-K decision; 0 = never split (test hook)
// split-K target workgroups (hconv and the persistent hconv3): 256 = one per CU. 512 (two per CU)
// split the 8x8 / 4x4 / 16x16 layers twice as often: more fp32 partials and last-arriver merges
// for no extra overlap. bench.py img/s, 512 -> 256 (profiles/split_target_r4.md): ResNet-18 b64
// 32.3k -> 35.0k, b128 54.2k -> 57.7k, b256 81.8k -> 83.5k; ResNet-50 b256 26.1k -> 26.2k, b32
// 7.85k -> 7.82k.
static int g_split_target = 256;
static int g_split_min_work = 4;  // taps x 64-channel chunks a split keeps at least
int hconv_split_target() { return g_split_target; }
void hconv_set_split_target(int t) { g_split_target = t < 0 ? 0 : t; }
void hconv_set_split_min_work(int w) { g_split_min_work = w < 1 ? 1 : w; }

int hconv_tiles(int NB, int H, int W, int Cs, int N, int ntaps) {
  H3Plan pl;
  if (hconv3_plan(NB, H, W, Cs, N, ntaps, &pl)) return pl.tiles_m * pl.tiles_n;
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  return (NB * H * W + bm - 1) / bm * ((N + bn - 1) / bn);
}

int hconv_tile_elems(int NB, int H, int W, int Cs, int N, int ntaps) {
  H3Plan pl;
  if (hconv3_plan(NB, H, W, Cs, N, ntaps, &pl)) return 16384;  // 4 waves x 64 x 64
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  return bm * bn;
}

// split-K factor: double while the grid is below the target (about two workgroups per CU), the
// 64-channel chunks still divide evenly and every split keeps at least 4 taps x chunks of work
int hconv_splits(int NB, int H, int W, int Cs, int N, int ntaps) {
  if (!hconv_supported(NB, H, W, Cs, N, ntaps)) return 1;
  H3Plan pl;
  if (hconv3_plan(NB, H, W, Cs, N, ntaps, &pl)) return pl.splits;
  const long tiles = hconv_tiles(NB, H, W, Cs, N, ntaps);
  const int nchunk = Cs / 64, target = hconv_split_target();
  int s = 1;
  while (target > 0 && tiles * s < target && nchunk % (2 * s) == 0 && (nchunk / (2 * s)) * ntaps >= g_split_min_work) s *= 2;
  return s;
}

bool hconv_v3(int NB, int H, int W, int Cs, int N, int ntaps) {
  H3Plan pl;
  return hconv3_plan(NB, H, W, Cs, N, ntaps, &pl);
}

int hconv_stat_rows(int NB, int H, int W, int Cs, int N, int ntaps, int f32out) {
  H3Plan pl;  // (fp32-output launches stay on hconv_kernel)
  if (!f32out && hconv3_plan(NB, H, W, Cs, N, ntaps, &pl)) return pl.tiles_m;
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  return (NB * H * W + bm - 1) / bm;
}

template <int BM, int BN, bool F32O>
static void launch_hconv(HConvArgs a, hipStream_t s) {
  if (!hconv_geometry(a.NB, a.H, a.W, BM, &a.TH, &a.TW, &a.IMG)) throw std::runtime_error("hconv: bad geometry");
  const long mt = (long)(a.NB / a.IMG) * (a.H / a.TH) * (a.W / a.TW);
  const int grid = (int)(mt * ((a.N + BN - 1) / BN));
  const int hp = a.IMG * (a.TH + 2) * (a.TW + 2);
  a.HPR = ((hp + 31) / 32) * 32;  // halo buffer sized to the tile (LDS decides workgroups per CU)
  const bool multi = a.Cs / 64 / a.splits > 1;  // >1 channel chunk per workgroup: double-buffered halo
  // taps per K step. Default: 2 on the 64x64 tiles (small maps, long K: 4x4 layer-4 convs 9%
  // faster, same workgroups per CU), 1 elsewhere (2 or 3 cost a resident workgroup per CU on the
  // larger tiles: 20-40% slower, tools/gpu_exp.sh sweep in profiles/experiment_hconv_variants.md)
  const int tps = (BM == 64 && BN == 64 && a.ntaps >= 4) ? 2 : 1;
  constexpr int bstages = 3;
  // deep weight ring: one tap per step, every halo prefetch >= NBS steps ahead of its use, and
  // only where the extra stage keeps the workgroups per CU (LDS-bound occupancy: losing one
  // costs more than the deeper prefetch gains, measured 63.4k vs 65.0k img/s on ResNet-18)
  auto wg_per_cu = [&](int nb) {
    const int main = (multi ? 2 : 1) * a.HPR * 128 + nb * BN * 128, epi = BM * (BN * (F32O ? 4 : 2) + 16);
    return 163840 / (main > epi ? main : epi);
  };
  int nbs = (tps == 1 && a.ntaps >= bstages) ? bstages : 2;
  while (nbs > 2 && wg_per_cu(nbs) < wg_per_cu(2)) --nbs;
#define DCNN_HC(TPS, NHB, NBS)                                                                         \
  {                                                                                                    \
    auto k = hconv_kernel<BM, BN, TPS, NHB, NBS, F32O>;                                                \
    const int lds = HC<BM, BN, TPS, NHB, NBS, F32O>::lds_bytes(a.HPR * 128);                           \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(grid * a.splits), dim3(256), lds, s, a);                                \
  }
  if (tps == 2) {
    if (multi) DCNN_HC(2, 2, 2) else DCNN_HC(2, 1, 2)
  } else if (nbs == 3) {
    if (multi) DCNN_HC(1, 2, 3) else DCNN_HC(1, 1, 3)
  } else {
    if (multi) DCNN_HC(1, 2, 2) else DCNN_HC(1, 1, 2)
  }
#undef DCNN_HC
  DCNN_LAUNCH_CHECK();
}

void hconv(HConvArgs a, hipStream_t s) {
  if (!hconv_supported(a.NB, a.H, a.W, a.Cs, a.N, a.ntaps)) throw std::runtime_error("hconv: unsupported shape");
  for (int t = 0; t < a.ntaps; ++t)
    if (a.tap_dy[t] < -1 || a.tap_dy[t] > 1 || a.tap_dx[t] < -1 || a.tap_dx[t] > 1)
      throw std::runtime_error("hconv: taps must reach at most 1 pixel");
  if (a.splits < 1) a.splits = 1;
  if (a.splits != 1 && (a.splits != hconv_splits(a.NB, a.H, a.W, a.Cs, a.N, a.ntaps) || !a.part || !a.tickets))
    throw std::runtime_error("hconv: split count / workspace mismatch (use hconv_splits)");
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  if (!a.Cf && hconv3_try(a, s)) return;
  if (a.Cf) {
    if (a.bnb.x) throw std::runtime_error("hconv: no backward-BN fusion with fp32 output");
    if (bm == 128 && bn == 128) return launch_hconv<128, 128, true>(a, s);
    if (bm == 128 && bn == 64) return launch_hconv<128, 64, true>(a, s);
    if (bm == 64 && bn == 128) return launch_hconv<64, 128, true>(a, s);
    return launch_hconv<64, 64, true>(a, s);
  }
  if (bm == 128 && bn == 128) return launch_hconv<128, 128, false>(a, s);
  if (bm == 128 && bn == 64) return launch_hconv<128, 64, false>(a, s);
  if (bm == 64 && bn == 128) return launch_hconv<64, 128, false>(a, s);
  return launch_hconv<64, 64, false>(a, s);
}

}  // namespace dcnn
