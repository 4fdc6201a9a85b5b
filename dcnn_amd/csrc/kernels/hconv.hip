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
//             for each tap t: B(c, t) [prefetched one step ahead], MFMA over 64 channels
//
// The epilogue is the gemm2 one (bias, residual, ReLU, BatchNorm partial statistics, 16-byte
// stores through an LDS-staged bf16 tile), with the spatial-tile -> NHWC row mapping.
#include "common.h"
#include "api.h"

namespace dcnn {

typedef __attribute__((address_space(3))) void lds_void_h;

namespace {
constexpr unsigned kOOBh = 0x80000000u;

__device__ __forceinline__ void glds16h(__amdgpu_buffer_rsrc_t rsrc, char* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_h*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int xcd_remap_h(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// 128-byte LDS rows (64 bf16 channels), 16-byte chunks XOR-swizzled by the row's low 3 bits
__device__ __forceinline__ int hoff(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }
}  // namespace

// TPS taps per K step (one barrier per step), NHB halo buffers (1 when there is a single
// 64-channel chunk: nothing to prefetch)
template <int BM, int BN, int TPS, int NHB>
struct HC {
  static constexpr int TM = BM / 32, TN = BN / 32;      // 16x16 subtiles per wave (2x2 waves)
  static constexpr int BTAP = BN * 128;                  // bytes of one tap's weight slice
  static constexpr int BST = TPS * BTAP;                 // bytes per weight stage
  static constexpr int B_INS = BN / 32;                  // glds per wave per tap slice
  static constexpr int EPI_PITCH = BN * 2 + 16;
  // dynamic LDS: NHB halo buffers of HALO = 128 * (halo rows padded to 32) bytes, then 2 weight stages
  static int lds_bytes(int halo) {
    const int main = NHB * halo + 2 * BST, epi = BM * EPI_PITCH;
    return main > epi ? main : epi;
  }
};

template <int BM, int BN, int TPS, int NHB>
__global__ void __launch_bounds__(256, 1) hconv_kernel(HConvArgs p) {
  using T = HC<BM, BN, TPS, NHB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  struct { int HALO; } T_rt{p.HPR * 128};
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = p.N / BN;
  const int lt = xcd_remap_h(blockIdx.x, gridDim.x);
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

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.b_bytes, 0x00020000);

  // ---- halo loader: per-lane pixel base offsets for its rows (fixed across chunks) ----
  const int hch = lane & 7;                               // physical chunk slot
  const int HNI = (HP + 31) / 32;                         // glds per wave per halo chunk (8 rows each)
  unsigned h_base[10];
  int h_row[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {
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
    for (int j = 0; j < 10; ++j) {
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
    const int m = wm * (BM / 2) + i * 16 + (lane & 15);   // tile-local output row
    const int tpx = p.TH * p.TW;
    const int im = m / tpx, r2 = m - im * tpx;
    arow0[i] = im * HPI + (r2 / p.TW + 1) * HW2 + (r2 % p.TW + 1);
  }

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunk = p.Cs / 64;
  const int spc = (p.ntaps + TPS - 1) / TPS;  // K steps per channel chunk
  const int nsteps = nchunk * spc;
  load_halo(0, 0);
  load_b(0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int bcur = 0;
  for (int k = 0; k < nsteps; ++k) {
    const int c = k / spc, t0 = (k - c * spc) * TPS;
    if (k + 1 < nsteps) {
      const int c1 = (k + 1) / spc, t1 = (k + 1 - c1 * spc) * TPS;
      load_b(bcur ^ 1, c1 * 64, t1);
      if (NHB == 2 && t0 == 0 && c + 1 < nchunk) load_halo((c + 1) & 1, (c + 1) * 64);
    }
    const char* Hs = smem + (NHB == 2 ? (c & 1) : 0) * T_rt.HALO;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int t = t0 + u;
      if (TPS > 1 && t >= p.ntaps) break;
      const char* Bs = smem + NHB * T_rt.HALO + bcur * T::BST + u * T::BTAP;
      const int toff = p.tap_dy[t] * HW2 + p.tap_dx[t];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
        bf16x8 a[T::TM], b[T::TN];
#pragma unroll
        for (int i = 0; i < T::TM; ++i) a[i] = *reinterpret_cast<const bf16x8*>(Hs + hoff(arow0[i] + toff, ch));
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(Bs + hoff(wn * (BN / 2) + j * 16 + (lane & 15), ch));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < T::TM; ++i)
#pragma unroll
          for (int j = 0; j < T::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bcur ^= 1;
  }

  // ---- epilogue 1: acc (+bias) -> bf16 LDS tile [BM][BN] ----
#pragma unroll
  for (int j = 0; j < T::TN; ++j) {
    const int col = wn * (BN / 2) + j * 16 + (lane & 15);
    const float bv = p.bias ? p.bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        *reinterpret_cast<bf16*>(smem + row * T::EPI_PITCH + col * 2) = (bf16)(acc[i][j][r] + bv);
      }
  }
  __syncthreads();
  // ---- epilogue 2: 16-byte rows -> NHWC global (+residual, ReLU, BN partial stats) ----
  constexpr int CG = BN / 8;
  constexpr int RSTEP = 256 / CG;
  const int cg = tid % CG, r0 = tid / CG;
  const int ncol = n0 + cg * 8;
  float s[8], q[8], mu[8], is[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) s[v] = q[v] = mu[v] = is[v] = 0.f;
  const bool bnb = p.bnb.x != nullptr;  // backward-BN fusion (api.h BnbArgs)
  if (bnb && true) {
#pragma unroll
    for (int v = 0; v < 8; ++v) { mu[v] = p.bnb.mean[ncol + v]; is[v] = p.bnb.istd[ncol + v]; }
  }
  const int tpx = p.TH * p.TW;
  for (int row = r0; row < BM; row += RSTEP) {
    const int im = row / tpx, r2 = row - im * tpx;
    const int n = img0 + im;
    if (n >= p.NB) continue;
    const long orow = ((long)n * p.H + y0 + r2 / p.TW) * p.W + x0 + r2 % p.TW;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(smem + row * T::EPI_PITCH + cg * 16), f);
    if (p.residual) {
      float rr[8];
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
    const uint4 o = pack8(f);
    *reinterpret_cast<uint4*>(p.C + orow * p.N + ncol) = o;
    if (p.stats) {
      float g[8];
      unpack8(o, g);
      if (bnb) {
        float xv[8];
        unpack8(*reinterpret_cast<const uint4*>(p.bnb.x + orow * p.N + ncol), xv);
#pragma unroll
        for (int v = 0; v < 8; ++v) { s[v] += g[v]; q[v] += g[v] * (xv[v] - mu[v]) * is[v]; }
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v) { s[v] += g[v]; q[v] += g[v] * g[v]; }
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
    for (int cc = tid; cc < 2 * BN; cc += 256) {
      const int which = cc / BN, c2 = cc % BN;
      float a = 0.f;
      for (int k = 0; k < RSTEP; ++k) a += red[(k * 2 + which) * BN + c2];
      p.stats[((long)tm * 2 + which) * p.N + n0 + c2] = a;
    }
  }
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
  if ((img * (th + 2) * (tw + 2)) > 320) return false;
  *TH = th; *TW = tw; *IMG = img;
  (void)NB;
  return true;
}

static void hconv_pick(const HConvArgs& a, int* bm, int* bn) {
  // prefer 128 x 128 when it still gives >= ~1.5 workgroups per CU, else shrink
  auto tiles = [&](int m, int n) { return (long)((a.NB * a.H * a.W + m - 1) / m) * (a.N / n); };
  *bm = 128;
  *bn = (a.N % 128 == 0 && tiles(128, 128) >= 384) ? 128 : 64;
  if (tiles(*bm, *bn) < 384) *bm = 64;
}

bool hconv_supported(int NB, int H, int W, int Cs, int N, int ntaps) {
  if (Cs % 64 || N % 64 || ntaps < 1 || ntaps > 9) return false;
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn, th, tw, img;
  hconv_pick(a, &bm, &bn);
  if (!hconv_geometry(NB, H, W, bm, &th, &tw, &img)) return false;
  return NB % img == 0;
}

int hconv_stat_rows(int NB, int H, int W, int N) {
  HConvArgs a{};
  a.NB = NB; a.H = H; a.W = W; a.N = N;
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  return (NB * H * W + bm - 1) / bm;
}

template <int BM, int BN>
static void launch_hconv(HConvArgs a, hipStream_t s) {
  if (!hconv_geometry(a.NB, a.H, a.W, BM, &a.TH, &a.TW, &a.IMG)) throw std::runtime_error("hconv: bad geometry");
  const long mt = (long)(a.NB / a.IMG) * (a.H / a.TH) * (a.W / a.TW);
  const int grid = (int)(mt * (a.N / BN));
  const int hp = a.IMG * (a.TH + 2) * (a.TW + 2);
  a.HPR = ((hp + 31) / 32) * 32;  // halo buffer sized to the tile (LDS decides workgroups per CU)
  const bool multi = a.Cs > 64;
  static const int tps = [] {
    const char* e = getenv("DCNN_HCONV_TPS");
    return (e && atoi(e) == 3) ? 3 : 1;  // 3 taps/step: fewer barriers but 1 workgroup/CU (slower)
  }();
#define DCNN_HC(TPS, NHB)                                                                              \
  {                                                                                                    \
    auto k = hconv_kernel<BM, BN, TPS, NHB>;                                                           \
    const int lds = HC<BM, BN, TPS, NHB>::lds_bytes(a.HPR * 128);                                      \
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, s, a);                                           \
  }
  if (tps == 3) {
    if (multi) DCNN_HC(3, 2) else DCNN_HC(3, 1)
  } else {
    if (multi) DCNN_HC(1, 2) else DCNN_HC(1, 1)
  }
#undef DCNN_HC
  DCNN_LAUNCH_CHECK();
}

void hconv(HConvArgs a, hipStream_t s) {
  if (!hconv_supported(a.NB, a.H, a.W, a.Cs, a.N, a.ntaps)) throw std::runtime_error("hconv: unsupported shape");
  for (int t = 0; t < a.ntaps; ++t)
    if (a.tap_dy[t] < -1 || a.tap_dy[t] > 1 || a.tap_dx[t] < -1 || a.tap_dx[t] > 1)
      throw std::runtime_error("hconv: taps must reach at most 1 pixel");
  int bm, bn;
  hconv_pick(a, &bm, &bn);
  if (bm == 128 && bn == 128) return launch_hconv<128, 128>(a, s);
  if (bm == 128 && bn == 64) return launch_hconv<128, 64>(a, s);
  if (bm == 64 && bn == 128) return launch_hconv<64, 128>(a, s);
  return launch_hconv<64, 64>(a, s);
}

}  // namespace dcnn
