// Launcher API of the dcnn_amd HIP kernel library (shared by the .hip TUs and the bindings).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fusion_plan.h"  // the shared fusion planner (both front ends)
typedef __bf16 bf16;

namespace dcnn {
// Backward-BatchNorm fusion into a dgrad epilogue. The GEMM output is the gradient arriving at
// a BatchNorm(+ReLU) layer: the epilogue masks it with that layer's ReLU output (y > 0, when y
// is set), stores the masked gradient dy', and writes per-tile (sum dy', sum dy' * xhat) rows
// into `stats`, xhat = (x - mean) * istd — the statistics the BN backward needs, without a
// separate pass over dy, x and y. Inactive when x == nullptr.
struct BnbArgs {
  const bf16* y; const bf16* x; const float* mean; const float* istd;
  // mask_x (hconv3's data-gradient epilogue only; the other kernels use y): the ReLU mask
  // recomputed from x as the forward apply computed it, x * (gamma istd) + (beta - mean gamma
  // istd) > 0, instead of read from y (a plain BatchNorm + ReLU; gamma / beta null: no affine)
  const float* gamma; const float* beta; int mask_x;
};
struct NtArgs {
  const bf16* A; const bf16* B; void* C;
  int M, N, K; int lda, ldb, ldc; int mode;
  int nb, sh, sw, cs, gh, gw; int kh, kw, strh, strw, padh, padw;
  const float* bias; const bf16* residual; float* stats; int out_f32; int relu;
};
struct TnArgs {
  const bf16* dY; const bf16* X; float* slab; float* bias_slab;
  int M, N, P; int mode; int nb, sh, sw, cs, gh, gw; int kh, kw, strh, strw, padh, padw; int ldx; int k_per_split;
};
struct G2Args {
  const bf16* A; const bf16* B; bf16* C;
  unsigned a_bytes, b_bytes;
  int M, N, Cs, H, W, GH, GW, SY, SX, ntaps;
  int tap_dy[64], tap_dx[64], tap_srcoff[64], tap_b[64];
  int ldb, ldc;
  int OH, OW, OSY, OSX, ORY, ORX;
  const float* bias; const bf16* residual; float* stats; int relu;
  float* zero_ptr; int zero_n;  // zeroed by workgroup 0 (BN sums consumed by the next kernel)
  BnbArgs bnb;
  // grouped launch of up to 4 row classes (the stride phases of a strided dgrad): class c owns
  // rows [c * cls_rows, (c + 1) * cls_rows) (cls_rows a multiple of the row tile), taps
  // [cls_t0[c], cls_t0[c] + cls_nt[c]) of the tap arrays and the output phase (cls_ory, cls_orx).
  // ncls <= 1: the single class (taps 0..ntaps-1, ORY/ORX), filled in by gemm_g2().
  int ncls, cls_rows;
  int cls_t0[4], cls_nt[4], cls_ory[4], cls_orx[4];
  // split-K (set by gemm_g2() for long-K 1x1 GEMMs on small grids): K slices, fp32 partials
  int ksplit; float* kpart;
  // multiply-shift reciprocals of GH * GW and GW (set by gemm_g2(): the per-row pixel decode of
  // the A loader and the epilogue without run-time integer divisions; common.h FastDiv layout)
  unsigned fd_ghw[3], fd_gw[3];
};
struct T2Args {
  const bf16* dY; const bf16* X; float* slab; float* bias_slab;
  unsigned a_bytes, b_bytes;
  int M, N, P, ldy, Cs, H, W, GH, GW, SY, SX, ntaps;
  int tap_dy[64], tap_dx[64];
  int k_per_split;
};
struct PoolGeom { int N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw; };
// NHWC conv geometry of the explicit im2col path (im2col.hip)
struct ConvGeom { int N, H, W, C, OH, OW, KH, KW, SH, SW, PH, PW; };
// halo-tiled stride-1 direct conv (hconv.hip): out[NB][H][W][N] = sum_t in[y+dy_t][x+dx_t][:] . B[n][tap_b_t + :]
struct HConvArgs {
  const bf16* A; const bf16* B; bf16* C;
  unsigned a_bytes, b_bytes;
  int NB, H, W, Cs, N, ldb, ntaps;
  int tap_dy[9], tap_dx[9], tap_b[9];
  int TH, TW, IMG, HPR;  // filled by the launcher (HPR: halo rows padded to 32)
  const float* bias; const bf16* residual; float* stats; int relu;
  float* zero_ptr; int zero_n;  // zeroed by workgroup 0 (BN sums accumulated by the next kernel)
  BnbArgs bnb;
  // fp32 output (split-precision fp32 convs, ops/hip.py): when Cf is set the result (+ the fp32
  // residual residual_f) is written to Cf as fp32 instead of C as bf16 (no backward-BN fusion)
  float* Cf; const float* residual_f;
  // split-K over 64-channel chunks (small grids): `splits` workgroups per output tile, partial
  // accumulators in `part` [tiles][splits][BM*BN] fp32, the last arriver on the tile's ticket
  // word sums them in split order (deterministic) and runs the epilogue; tickets left zeroed
  int splits; float* part; unsigned* tickets;
};
void hconv(HConvArgs a, hipStream_t s);
// split count hconv() will use for this shape, and its output-tile count (workspace sizing)
int hconv_splits(int NB, int H, int W, int Cs, int N, int ntaps);
int hconv_tiles(int NB, int H, int W, int Cs, int N, int ntaps);
int hconv_tile_elems(int NB, int H, int W, int Cs, int N, int ntaps);
int hconv_split_target();
void gemm_t2_set_split_target(int t);  // test / tuning hook (default 512)
void hwgrad_set_split_target(int t);   // test / tuning hook (default 256)
void hconv3_set_max_splits(int n);     // tuning hook (default 8)
void g1s_set_waves_per_simd(int w);    // tuning hook (default 2)
void hconv_set_split_target(int t);  // workgroups the split-K decision aims for (0: never split)
void hconv_set_split_min_work(int w);  // least taps x 64-channel chunks per split (default 4)
void bn_set_vectorised(int on);   // bf16 BatchNorm apply passes on the vectorised kernels (default on)
bool hconv_supported(int NB, int H, int W, int Cs, int N, int ntaps);
int hconv_stat_rows(int NB, int H, int W, int Cs, int N, int ntaps, int f32out);
// exact fp32 on the persistent halo conv (hconv3.hip F32 instances): A / B fp32 through the pointer
// fields, Cs fp32 input channels, ldb / tap_b in fp32 elements, output Cf (+ residual_f), statistics
// / bias / ReLU as hconv; false = not covered (nothing launched). Split-K workspace as hconv with
// hconv3_f32_splits (0: not covered); statistics rows = the tile count (hconv3_f32_tiles).
bool hconv3_f32_try(const HConvArgs& a, hipStream_t s);
int hconv3_f32_splits(int NB, int H, int W, int Cs, int N, int ntaps);
bool hconv_v3(int NB, int H, int W, int Cs, int N, int ntaps);  // shape runs on hconv3
void hconv3_enable(int on);
void hconv3_set_grid_cap(int n);      // test hook: cap the persistent grid (0: resident workgroups)
void hconv3_set_stamps(uintptr_t p);  // diagnostic per-item timeline buffer (u64 [items][4][16]) or 0
// halo-tiled stride-1 weight gradient (hwgrad.hip): slab[split][Co][t*Cs + c] = partial dW
struct HWArgs {
  const bf16* dY; const bf16* X; float* slab; float* bias_slab;  // bias_slab[split][Co] (optional)
  unsigned dy_bytes, x_bytes;
  int NB, H, W, Cs, Co, ntaps;
  int tap_dy[9], tap_dx[9];
  int TH, TW, IMG, HPR, tiles_per_split;  // filled by the launcher
  // operand pairs (grid.y): pair q reads dY channels [yoff_q, yoff_q + Co) of rows ldy wide and
  // X channels [xoff_q, xoff_q + Cs) of rows ldx wide, into slabs [q * splits + split]; its bias
  // partial is the dY column sum if bias_q else 0. One pair with ldy = Co, ldx = Cs is the plain
  // wgrad; three over [hi|lo|hi] rows are the split-precision fp32 one (ops/hip.py).
  int ldy, ldx, npairs;
  int pair_yoff[3], pair_xoff[3], pair_bias[3];
};
void hwgrad(HWArgs a, int splits, hipStream_t s);
bool hwgrad_supported(int NB, int H, int W, int Cs, int Co, int ntaps);
int hwgrad_splits(int NB, int H, int W, int Cs, int Co);
// exact fp32 halo weight gradient (3x3 pad-1 stride-1): dY / X fp32 through HWArgs' pointer fields,
// Cs / Co fp32 channels (multiples of 32), slab [splits][Co][9 Cs]
bool hwgrad_f32_supported(int NB, int H, int W, int Cs, int Co);
int hwgrad_f32_splits(int NB, int H, int W, int Cs, int Co);
void hwgrad_f32(HWArgs a, int splits, hipStream_t s);
void hwgrad_set_version(int v);  // 2: tap-shift-invariant kernel where it applies, 1: first kernel
// halo weight gradient of a 3x3 / stride-2 / pad-1 conv (hwgrad.hip): dY H x W (the output grid), X
// 2H x 2W, plain operands (ldy = Co, ldx = Cs), slab [splits][Co][9 Cs] (+ bias_slab [splits][Co])
bool hwgrad_s2_supported(int NB, int H, int W, int Cs, int Co);
int hwgrad_s2_splits(int NB, int H, int W, int Cs, int Co);
void hwgrad_s2(HWArgs a, int splits, hipStream_t s);

void gemm_nt(const NtArgs& a, hipStream_t s);
void gemm_g2(const G2Args& a, hipStream_t s);
// split-K for long-K (>= 1024) 1x1 GEMMs on small grids: K slices to fp32 partials + an epilogue
// launch (default on; 0: the routing table keeps those convs on the halo kernel)
void gemm_g2_set_splitk(int on);
int gemm_g2_splitk_enabled();
int gemm_g2_stat_rows(int M, int N);
int gemm_g2_row_tile(int M, int N);  // BM the launcher picks for an M x N output
void gemm_t2(T2Args a, int splits, hipStream_t s);
// streaming 1x1 conv (g1s.hip): mode 0 plain, 1 forward + Welford statistics, 2 dgrad + bnb sums
int g1s_rows(int M, int N, int K, int mode);
void g1s_enable(int on);
void g1s(const bf16* X, const bf16* Wt, bf16* Y, int M, int N, int K, int H, int W, int OH, int OW, int S,
         const float* bias, const bf16* residual, float* stats, int relu, float* zero_ptr, int zero_n, BnbArgs bnb,
         int mode, hipStream_t s);
int g1s_gen_rows(int M, int N, int Kc, int ntaps, int mode);
void g1s_gen(const bf16* X, const bf16* Wt, bf16* Y, int NB, int GH, int GW, int N, int Kc, int ldw,
             const std::vector<std::array<int, 3>>& taps, int H, int W, int OHo, int OWo, int OS, int ORY, int ORX,
             const bf16* residual, float* stats, float* zero_ptr, int zero_n, BnbArgs bnb, int mode, hipStream_t s);
int gemm_t2_splits(int M, int N, int P);
int gemm_nt_stat_rows(int M, int N);
// generic tensor ops (ops.hip)
void elementwise(int mode, int op, const float* a, const float* b, float* c, long n, float s0, float s1, hipStream_t s);
void reduce(int op, const float* a, const float* b, long n, float* workspace, float* out, hipStream_t s);
void fill_random(float* out, long n, uint64_t seed, float a, float b, int normal, hipStream_t s);
void transpose_batched(const float* in, float* out, int batch, int rows, int cols, hipStream_t s);
void transpose_batched16(const void* in, void* out, int batch, int rows, int cols, hipStream_t s);
void rows_copy(int kind, const void* src, int lds, void* dst, int ldd, long rows, int cols, hipStream_t s);
void nchw_cnhw(const float* in, float* out, int N, int C, int HW, int to_cnhw, hipStream_t s);
void pad_crop(const float* in, float* out, int NC, int H, int W, int OH, int OW, int top, int left, float value,
              hipStream_t s);
// fp32 path (gemm_f32.hip): same argument structs, fp32 operand/result pointers
void gemm_g2f(const G2Args& a, hipStream_t s);
int gemm_g2f_stat_rows(int M, int N);
void gemm_t2f(T2Args a, int splits, hipStream_t s);
int gemm_t2f_splits(int M, int N, int P);
void set_f32_mode(int mode);  // 0 exact f32 MFMA (default), 1 split-bf16 (3 MFMAs)
int get_f32_mode();
void conv_weight_transpose_f32(const float* w, float* wt, int Co, int T_, int Ci, hipStream_t s);
void gemm_tn(TnArgs a, int splits, hipStream_t s);
int gemm_tn_splits(int M, int N, int P);
// The shared conv routing table (conv_route.cpp): which kernel family runs a bf16 convolution,
// asked by both front ends (ops/hip.py and the C++ host API's GPU backend). g1s_mode: the
// streaming kernel's epilogue mode the caller needs (forward 0 / 1 = statistics, dgrad 0 / 2 =
// backward-BatchNorm fusion), < 0 when the epilogue options rule it out.
struct ConvRouteGeom {
  int N, C, H, W, Co, KH, KW, SH, SW, PH, PW, OH, OW, g1s_mode;
};
enum ConvRoute : int { ROUTE_GENERIC = 0, ROUTE_GEMM_G2 = 1, ROUTE_HALO = 2, ROUTE_G1S = 3, ROUTE_HALO_S2 = 4 };
int conv_fwd_route(ConvRouteGeom g);
int conv_dgrad_route(ConvRouteGeom g);
int conv_wgrad_route(ConvRouteGeom g);
// (the shared fusion planner: fusion_plan.h, included above)
void splitk_reduce(const float* slab, float* out, long n, int splits, int accumulate, hipStream_t s);
// weight + bias slabs in one launch (nb = 0: bias segment absent)
void splitk_reduce2(const float* slab, float* out, long n, const float* bslab, float* bout, long nb, int splits,
                    int accumulate, hipStream_t s);

// many split-K slab reductions in one launch (grad += sum over splits), kernel-argument table
constexpr int kMaxRed = 48;
struct RedEnt { const float* slab; float* out; long n; int splits, unit0, chunks, groups, vec, wpc; };  // wpc: waves per chunk
struct MultiRed { int count; RedEnt e[kMaxRed]; };
void multi_splitk_reduce(MultiRed t, hipStream_t s);

int bn_partial_rows(long R, int C);
void bn_partial(int dtype, const void* x, const void* dy, const void* yout, void* dy_out, const float* mean,
                const float* istd, long R, int C, float* slab, int mode, float* zero_sums, hipStream_t s);
// deterministic slab reduce: mode 0 Welford triples [rows][3][C] -> (mean, var); mode 1 sums [rows][2][C]
int bn_stat_parts(int rows);
// two independent reduces of the same C in one launch (segment 2 optional: slab2 = nullptr)
void bn_stat_reduce2(int mode, const float* slab, int rows, float* out, float* part, const float* slab2, int rows2,
                     float* out2, float* part2, int C, hipStream_t s);
void bn_stat_reduce(int mode, const float* slab, int rows, int C, float* out, float* part, unsigned* ticket,
                    hipStream_t s);
void bn_apply(int dtype, const void* x, void* y, long R, int C, const float* sums, int parts, float count, const float* gamma,
              const float* beta, float eps, const void* residual, int relu, float* save_mean, float* save_istd,
              float* run_mean, float* run_var, float momentum, int use_running, hipStream_t s);
// one BatchNorm's operands for bn_apply_dual (statistics as bn_apply: sums/parts or running)
struct BnSide {
  const void* x; const float* sums; int parts; float count; const float* gamma; const float* beta; float eps;
  float* save_mean; float* save_istd; float* run_mean; float* run_var; float momentum; int use_running;
};
// y = act(bn_a(a.x) + bn_b(b.x)): a residual block's tail BatchNorm with its projection
// shortcut's BatchNorm applied on the fly (bf16, C % 8 == 0); false = unsupported, nothing launched
bool bn_apply_dual(const BnSide& a, const BnSide& b, void* y, long R, int C, int relu, hipStream_t s);
bool bn_apply_dual_supported(long R, int C);
// one BatchNorm of bn_bwd_apply_dual: input x, output dx, saved (mean, istd), backward sums
struct BnBwdSide {
  const void* x; void* dx; const float* mean; const float* istd; const float* gamma; const float* sums; int parts;
  float count; float* dgamma; float* dbeta;
};
// dx_a, dx_b of two BatchNorms fed the same gradient dy, one pass (bf16, training statistics)
bool bn_bwd_apply_dual(const void* dy, const BnBwdSide& a, const BnBwdSide& b, long R, int C, hipStream_t s);
void bn_bwd_apply(int dtype, const void* dy, const void* yout, const void* x, void* dx, long R, int C, const float* mean,
                  const float* istd, const float* gamma, const float* sums, int parts, float count, float* dgamma,
                  float* dbeta, int eval_mode, hipStream_t s);
// training BatchNorm + ReLU + non-overlapping max-pool in one pass (stem), bf16 NHWC
bool bn_relu_maxpool_supported(PoolGeom g);
void bn_relu_maxpool(const bf16* x, bf16* y, uint8_t* idx, PoolGeom g, const float* sums, int parts, float count,
                     const float* gamma, const float* beta, float eps, float* save_mean, float* save_istd,
                     float* run_mean, float* run_var, float momentum, hipStream_t s);
void gn_fwd(int dtype, const void* x, void* y, int N, int HW, int C, int G, const float* gamma, const float* beta,
            float eps, float* save_mean, float* save_istd, hipStream_t s);
void gn_bwd(int dtype, const void* dy, const void* x, void* dx, int N, int HW, int C, int G, const float* gamma,
            const float* mean, const float* istd, float* dgamma, float* dbeta, float* aff, hipStream_t s);

void maxpool_fwd(int dt, const void* x, void* y, uint8_t* idx, PoolGeom g, hipStream_t s);
void maxpool_bwd(int dt, const void* dy, const uint8_t* idx, void* dx, PoolGeom g, hipStream_t s);
// max-pool backward fused with the producing BatchNorm+ReLU's backward statistics (stem)
bool maxpool_bwd_bnb_supported(PoolGeom g);
int maxpool_bwd_bnb_rows(PoolGeom g);
void maxpool_bwd_bnb(const bf16* dy, const uint8_t* idx, const bf16* ypool, const bf16* x, const float* mean,
                     const float* istd, bf16* dx, PoolGeom g, float* slab, float* zero_sums, hipStream_t s);
void avgpool_fwd(int dt, const void* x, void* y, PoolGeom g, hipStream_t s);
void avgpool_bwd(int dt, const void* dy, void* dx, PoolGeom g, hipStream_t s);
void act_fwd(int dt, const void* x, void* y, long n, int type, float a, hipStream_t s);
void act_bwd(int dt, const void* x, const void* dy, void* dx, long n, int type, float a, hipStream_t s);
void softmax_rows(int dt, const void* x, void* y, long rows, int C, hipStream_t s);
void softmax_rows_bwd(int dt, const void* y, const void* dy, void* dx, long rows, int C, hipStream_t s);
void dropout(int dt, const void* x, void* y, long n, float p, uint64_t seed, const uint64_t* ctr, hipStream_t s);
void counter_bump(uint64_t* ctr, uint64_t* slot, hipStream_t s);
void nchw_to_nhwc(int dt, const float* x, void* y, int N, int C, int HW, hipStream_t s);
void nchw_to_nhwc_pad(int dt, const float* x, void* y, int N, int C, int Cp, int HW, hipStream_t s);
void conv_weight_transpose(int src_dt, const void* w, bf16* wt, int Co, int T_, int Ci, hipStream_t s);
void cast_f32_bf16(const float* x, bf16* y, long n, hipStream_t s);
// RGB stem conv (stem.hip): 3x3 s1 p1 from fp32 NCHW input, Ci <= 4, Co in {16,32,48,64}
struct StemArgs {
  const float* x; const void* w; int w_bf16; long ws[4];  // weight [Co][Ci][3][3] element strides
  const float* bias; bf16* y; float* slab; float* zero_ptr; int zero_n;  // fwd
  const bf16* dy; float* bias_slab; long gs[4]; long n_slab;             // wgrad (gs: grad strides)
  int halo_bytes; int N, Ci, H, W, Co, TH;
  // wgrad with the stem BatchNorm's backward applied to dy on the fly (bn_x != nullptr: dy is that
  // BatchNorm's masked output gradient, bn_x its input): dy' = A dy + B (x - mean) + D per channel,
  // bn_bwd_apply_v_kernel's coefficients from the reduced sums (bn_sums / bn_parts, as
  // bn_stat_reduce leaves them); workgroup 0 adds the BatchNorm's parameter gradients
  const bf16* bn_x; const float* bn_mean; const float* bn_istd; const float* bn_gamma; const float* bn_sums;
  int bn_parts; float bn_count; float* bn_dgamma; float* bn_dbeta; int bn_eval;
};
bool stem_supported(int N, int Ci, int H, int W, int Co);
int stem_tiles_host(int N, int H, int W);
int stem_wgrad_blocks(int N, int H, int W);
int stem_wgrad_blocks_bnt(int N, int H, int W);  // (StemArgs::bn_x set)
void stem_fwd(StemArgs a, hipStream_t s);
void stem_wgrad(StemArgs a, int blocks, hipStream_t s);
// f32: fp32 operands (the exact fp32 path), else bf16
void multi_weight_transpose(const int64_t* table, int n, long max_tiles, hipStream_t s, int f32 = 0);
void im2col(const float* x, float* col, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW,
            int OH, int OW, hipStream_t s);
void col2im(const float* col, float* x, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH, int PW,
            int OH, int OW, hipStream_t s);
int loss_workspace_floats(int N);
void loss_fused(int dt, const void* pred, const float* target, const int64_t* labels, void* grad, float* loss_out,
                int* correct, int N, int C, int type, float param, float gscale, float* ws, unsigned* ticket,
                hipStream_t s);
void adam_step(float* p, const float* g, float* m, float* v, bf16* shadow, long n, float lr, float b1, float b2,
               float eps, float bc1, float bc2, float wd, int decoupled, const float* hyper, hipStream_t s);
void sgd_step(float* p, const float* g, float* vel, bf16* shadow, long n, float lr, float mom, const float* hyper,
              hipStream_t s);
void adam_scalars(float* hyper, float b1, float b2, hipStream_t s);
// data-parallel bf16 gradient wire format (comm.hip)
void grad_pack_bf16(const float* g, bf16* out, long n, float scale, hipStream_t s);
void grad_sum_chunks_bf16(const bf16* src, int w, long ld, long n, bf16* dst, hipStream_t s);
void grad_unpack_bf16(const bf16* in, float* g, long n, hipStream_t s);
void zero_bytes(void* p, long nbytes, hipStream_t s);
void copy_pair(void* d0, const void* s0, long n0, void* d1, const void* s1, long n1, hipStream_t s);
// fp32 rows [rows][C] -> bf16 [rows][3C]: pattern 0 = [hi | lo | hi], 1 = [hi | hi | lo]
// (hi = bf16(x), lo = bf16(x - hi)); a conv over the concatenations sums hi*hi + lo*hi + hi*lo
void split3_bf16(const float* in, bf16* out, long rows, int C, int pattern, hipStream_t s);
// explicit im2col conv path (im2col.hip; dt 0 fp32, 1 bf16): col [N*OH*OW][KH*KW*C] tap-major;
// col2im sums the taps of every input element (+ residual), chan_major: columns ordered (c, ky, kx)
void im2col_nhwc(int dt, const void* x, void* col, const ConvGeom& g, hipStream_t s);
void col2im_nhwc(int dt, const void* col, void* x, const void* residual, const ConvGeom& g, int chan_major,
                 hipStream_t s);
// device-side batch assembly + augmentation chain (augment.hip, data/device_loader.py)
enum { AUG_HFLIP = 0, AUG_VFLIP, AUG_ROTATION, AUG_BRIGHTNESS, AUG_CONTRAST, AUG_NOISE, AUG_CROP, AUG_CUTOUT,
       AUG_NORMALIZE };
constexpr int kAugMaxOps = 12;
constexpr int kAugMaxFloats = 16384;  // C*H*W staged in LDS (two fp32 buffers: 128 KB)
struct AugOpDev {
  int kind;
  float p;
  float a[6];  // op parameters (normalize: mean[3], std[3])
};
struct AugBatchArgs {
  const void* src;        // dataset [N][C][H][W], uint8 (x / 255) or fp32
  int src_u8;
  const int64_t* idx;     // [B] sample indices of this batch
  const int64_t* labels;  // [N] (nullptr: no label gather)
  int64_t* labels_out;    // [B]
  float* out;             // [B][C][H][W] fp32
  int B, C, H, W;
  unsigned long long seed;
  int nops;
  AugOpDev ops[kAugMaxOps];
};
bool augment_batch_supported(int C, int H, int W);
void augment_batch(const AugBatchArgs& a, hipStream_t s);
}  // namespace dcnn
