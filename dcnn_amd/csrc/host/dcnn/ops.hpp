// Device backends of the C++ host API's layers. The layer code (nn.cpp, plain C++) calls these;
// cpu_* run the native fp32 NCHW CPU kernels (csrc/native/cpu_ops.cpp, cpu_gemm.cpp), gpu_* the
// HIP/CDNA4 kernel library (csrc/kernels/*.hip) on bf16 NHWC activations with fp32 master
// parameters and bf16 operand shadows — the same kernels the Python front end launches.
#pragma once
#include <cstdint>

namespace dcnn {

struct ConvShape {
  int N, C, H, W, Co, KH, KW, SH, SW, PH, PW, OH, OW;
};
struct PoolShape {
  int N, C, H, W, OH, OW, KH, KW, SH, SW, PH, PW;
};
enum ActKind { ACT_RELU = 0, ACT_LEAKY_RELU = 1, ACT_ELU = 2, ACT_SIGMOID = 3, ACT_TANH = 4, ACT_LINEAR = 5 };

namespace cpu_ops {
void conv_fwd(const float* x, const float* w, const float* b, float* y, const ConvShape& s);
void conv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, const ConvShape& s);
void dense_fwd(const float* x, const float* w, const float* b, float* y, long N, long In, long Out);
void dense_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, long N, long In,
               long Out);
void bn_fwd(const float* x, float* y, long N, long C, long HW, const float* g, const float* b, float eps, bool train,
            float* rmean, float* rvar, float momentum, float* smean, float* sistd);
void bn_bwd(const float* x, const float* dy, const float* mean, const float* istd, const float* g, float* dx,
            float* dg, float* db, long N, long C, long HW, bool train);
void maxpool_fwd(const float* x, float* y, int32_t* idx, const PoolShape& p);
void maxpool_bwd(const float* dy, const int32_t* idx, float* dx, const PoolShape& p);
void avgpool_fwd(const float* x, float* y, const PoolShape& p);
void avgpool_bwd(const float* dy, float* dx, const PoolShape& p);
void act_fwd(int kind, const float* x, float* y, long n, float alpha);
void act_bwd(int kind, const float* x, const float* dy, float* dx, long n, float alpha);
double softmax_ce(const float* pred, const int64_t* labels, float* grad, long N, long C, long* correct);
// the six losses (kind: 0 ce, 1 softmax ce, 2 log-softmax ce, 3 mse, 4 mae, 5 huber); target
// [N][C] fp32 or null (then `labels` are one-hot targets)
double loss(int kind, const float* pred, const float* target, const int64_t* labels, float* grad, long N, long C,
            float param, long* correct);
void groupnorm_fwd(const float* x, float* y, long N, long C, long HW, long G, const float* g, const float* b, float eps,
                   float* smean, float* sistd);
void groupnorm_bwd(const float* x, const float* dy, const float* mean, const float* istd, const float* g, float* dx,
                   float* dg, float* db, long N, long C, long HW, long G);
void softmax_fwd(const float* x, float* y, long N, long C, long HW);
void softmax_bwd(const float* y, const float* dy, float* dx, long N, long C, long HW);
// inverted dropout with a counter-based mask of (seed, element index): the same call on dy
// applies the forward's mask in backward
void dropout(const float* x, float* y, long n, float p, uint64_t seed);
// residual join: y = a + b (+ ReLU); ReLU mask of a gradient by the join's output; dx = a + b
void add(const float* a, const float* b, float* y, long n, bool relu);
void relu_mask(const float* dy, const float* y, float* dx, long n);
void adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps, float bc1,
          float bc2, float wd, bool decoupled);
void sgd(float* p, const float* g, float* vel, long n, float lr, float momentum);
}  // namespace cpu_ops

namespace gpu_ops {
// weight-gradient partial reduces of a backward batched into one launch at its end
void begin_deferred_reduce();
void end_deferred_reduce();
// launch the weight-gradient reduces queued so far now and keep queueing (a gradient consumer
// inside the backward: the data-parallel bucket all-reduce)
void flush_deferred_reduce();
// test-only fault injection (capi.cpp): bit 0 = conv_dgrad drops the fused BatchNorm ReLU mask
void set_fault(int f);
// fp32 NCHW network input -> bf16 NHWC activation
void input_to_nhwc(const float* x, void* y, int N, int C, int HW);
// bf16 [N][HW][C] <-> [N][C][HW] (Flatten keeps the NCHW feature order of the reference)
void nhwc_to_nchw(const void* x, void* y, int N, int HW, int C);
void nchw_to_nhwc_bf16(const void* x, void* y, int N, int HW, int C);
void cast_bf16(const float* x, void* y, long n);
void zero(void* p, long nbytes);
// w: bf16 [Co][KH][KW][C]; bias fp32 or null
// stat_rows != nullptr: also the BatchNorm statistics of y ([rows][3][Co] Welford triples, in a
// workspace valid until the next conv_fwd / stem_fwd) from the conv's epilogue; returns the slab
// and sets *stat_rows (0 and nullptr when the route has no statistics epilogue)
const float* conv_fwd(const void* x, const void* w, const float* bias, void* y, const ConvShape& s,
                      int* stat_rows = nullptr);
// operands of the BatchNorm (+ ReLU) that produced a conv's input
struct BnbOperands {
  const void* y;  // the BN + ReLU output (ReLU mask; null: no ReLU)
  const void* x;  // the BN input
  const float* mean;
  const float* istd;
  // a plain BatchNorm + ReLU (no residual): the halo dgrad recomputes the mask from x, gamma,
  // beta instead of reading y (one full-resolution read fewer)
  const float* gamma = nullptr;
  const float* beta = nullptr;
  bool mask_from_x = false;
};
// residual: dx = dgrad + residual in the epilogue (a residual block's input gradient);
// w_transposed: w is already the [C][KH][KW][Co] dgrad operand (weight_transpose);
// bnb: the epilogue also masks dx with y > 0 and writes the producing BatchNorm's backward
// statistics ([rows][2][C] sums of dx' and dx' * xhat) — returns that slab (valid until the next
// conv_dgrad) and sets *bnb_rows; 0 / nullptr when the route has no such epilogue (dx is plain)
const float* conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, const void* residual = nullptr,
                        bool w_transposed = false, const BnbOperands* bnb = nullptr, int* bnb_rows = nullptr);
// [Co][T][C] bf16 -> [C][T][Co]; the batched form takes a device table of rows
// (src, dst, Co, T, C) and the largest 64x64-tile count per tap over the rows
void weight_transpose(const void* w, void* wt, int Co, int T, int C);
void multi_weight_transpose(const int64_t* table, int n, long max_tiles);
// gw fp32 [Co][KH][KW][C] and gb fp32 [Co] accumulate (+=); gb may be null
void conv_wgrad(const void* dy, const void* x, float* gw, float* gb, const ConvShape& s);
// the network's first conv straight from the fp32 NCHW input (RGB stem kernel: <= 4 input
// channels, 3x3 stride-1 'same', 16-multiple outputs up to 64); y bf16 NHWC
bool stem_ok(const ConvShape& s);
const float* stem_fwd(const float* x, const void* w, const float* bias, void* y, const ConvShape& s,
                      int* stat_rows = nullptr);
void stem_wgrad(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s);
// the stem's own BatchNorm backward folded into its weight gradient (that BatchNorm's input
// gradient is never materialised: the stem conv is its only consumer). dy is the BatchNorm's
// masked output gradient with its statistics rows in `slab` (bn_bwd_slab's operands); the
// BatchNorm's parameter gradients dg / db accumulate as bn_bwd_slab's do. Same result as
// bn_bwd_slab followed by stem_wgrad, bit for bit.
struct StemBn {
  const void* x;             // BatchNorm input (the stem conv's output), bf16 NHWC
  const float* mean;         // saved batch statistics
  const float* istd;
  const float* gamma;        // null: no affine
  float* dgamma;
  float* dbeta;
  const float* slab;         // backward statistics rows (sum dy, sum dy * xhat)
  int rows;
  bool train;
};
void stem_wgrad_bn(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s, const StemBn& bn);
// w: bf16 [Out][In]
void dense_fwd(const void* x, const void* w, const float* bias, void* y, int N, int In, int Out);
void dense_dgrad(const void* dy, const void* w, void* dx, int N, int In, int Out);
void dense_wgrad(const void* dy, const void* x, float* gw, float* gb, int N, int In, int Out);
// training: batch statistics (saved mean / istd, running stats updated); eval: running stats
// relu: y = max(bn(x) [+ residual], 0) in the same pass (a BatchNorm followed by a ReLU, or the
// tail BatchNorm of a residual block with the shortcut added)
void bn_fwd(const void* x, void* y, long R, int C, const float* g, const float* b, float eps, bool train,
            float* rmean, float* rvar, float momentum, float* smean, float* sistd, bool relu = false,
            const void* residual = nullptr);
// training statistics from a producer's slab (conv_fwd stat_rows) instead of a pass over x
void bn_fwd_slab(const void* x, void* y, long R, int C, const float* slab, int rows, const float* g, const float* b,
                 float eps, float* rmean, float* rvar, float momentum, float* smean, float* sistd, bool relu,
                 const void* residual = nullptr);
// backward from a consumer's statistics slab (conv_dgrad bnb: dy already masked)
void bn_bwd_slab(const void* dy, const void* x, void* dx, long R, int C, const float* mean, const float* istd,
                 const float* g, float* dg, float* db, bool train, const float* slab, int rows);
// yout: the forward output of a BatchNorm + ReLU (dy is masked with yout > 0); dy_out: the masked
// dy is also stored there (the shortcut branch of a residual block)
void bn_bwd(const void* dy, const void* x, void* dx, long R, int C, const float* mean, const float* istd,
            const float* g, float* dg, float* db, bool train, const void* yout = nullptr, void* dy_out = nullptr);
// ---- paired BatchNorms: a residual block's tail BatchNorm and its projection shortcut's
// BatchNorm share one apply pass forward (the shortcut's normalised output is never written) and
// one pass over the shared gradient backward; both statistics reduces run in one launch.
// While a SecondaryStats scope is alive on this thread, conv_fwd / stem_fwd write their statistics
// slab to a second workspace, so the shortcut conv's slab survives the main path's convs.
struct SecondaryStats {
  SecondaryStats();
  ~SecondaryStats();
};
// raw training statistics rows of x ([rows][3][C] Welford triples): the producer's slab when
// given, else a statistics pass over x into the secondary workspace
struct BnRaw {
  const float* slab;
  int rows;
};
BnRaw bn_stats_raw(const void* x, long R, int C, const float* slab, int rows);
struct BnFwdSide {
  const void* x;
  BnRaw raw;  // training only
  const float* g;
  const float* b;
  float eps;
  float* rmean;
  float* rvar;
  float momentum;
  float* smean;
  float* sistd;
};
bool bn_dual_ok(long R, int C);
// y = act(bn_a(a.x) + bn_b(b.x)): train = batch statistics of both sides (saved, running stats
// updated), else running statistics
void bn_fwd_dual(const BnFwdSide& a, const BnFwdSide& b, void* y, long R, int C, bool relu, bool train);
struct BnBwdSides {
  const void* x;
  void* dx;
  const float* mean;
  const float* istd;
  const float* g;
  float* dg;
  float* db;
};
// dx_a and dx_b of two training BatchNorms fed the same (already masked) gradient dy in one pass:
// a's backward statistics from a consumer slab (conv_dgrad bnb), b's from a statistics pass here
void bn_bwd_dual(const void* dy, const BnBwdSides& a, const float* slab_a, int rows_a, const BnBwdSides& b, long R,
                 int C);
// ---- training BatchNorm + ReLU + non-overlapping max-pool in one pass (the stem): the
// full-resolution output is never stored; statistics from the producer slab (or a pass over x)
bool bn_relu_maxpool_ok(const PoolShape& p);
void bn_relu_maxpool(const void* x, void* y, uint8_t* idx, const PoolShape& p, const float* slab, int rows,
                     const float* g, const float* b, float eps, float* rmean, float* rvar, float momentum,
                     float* smean, float* sistd);
// its backward: max-pool backward masked with ypool > 0, plus the BatchNorm's backward statistics
// slab (returned, *rows set) for bn_bwd_slab
const float* maxpool_bwd_bnb(const void* dy, const uint8_t* idx, const void* ypool, const void* x, const float* mean,
                             const float* istd, void* dx, const PoolShape& p, int* rows);
void maxpool_fwd(const void* x, void* y, uint8_t* idx, const PoolShape& p);
void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, const PoolShape& p);
void avgpool_fwd(const void* x, void* y, const PoolShape& p);
void avgpool_bwd(const void* dy, void* dx, const PoolShape& p);
void act_fwd(int kind, const void* x, void* y, long n, float alpha);
void act_bwd(int kind, const void* x, const void* dy, void* dx, long n, float alpha);
// pred / grad bf16 [N][C]; returns the mean loss, correct count in *correct
double softmax_ce(const void* pred, const int64_t* labels, void* grad, int N, int C, long* correct);
double loss(int kind, const void* pred, const float* target, const int64_t* labels, void* grad, int N, int C,
            float param, long* correct, float grad_scale = 1.f);
// the same without reading the value back: read_last_loss() after later work on the flow (a
// pipeline's last stage launches its backward first, then reads the loss once)
void loss_launch(int kind, const void* pred, const float* target, const int64_t* labels, void* grad, int N, int C,
                 float param, float grad_scale = 1.f);
double read_last_loss(long* correct);
// GroupNorm over bf16 NHWC rows [N][HW][C]
void groupnorm_fwd(const void* x, void* y, int N, int HW, int C, int G, const float* g, const float* b, float eps,
                   float* smean, float* sistd);
void groupnorm_bwd(const void* dy, const void* x, void* dx, int N, int HW, int C, int G, const float* g,
                   const float* mean, const float* istd, float* dg, float* db);
// softmax over the channels of every pixel (bf16 NHWC rows)
void softmax_fwd(const void* x, void* y, long rows, int C);
void softmax_bwd(const void* y, const void* dy, void* dx, long rows, int C);
void dropout(const void* x, void* y, long n, float p, uint64_t seed);
void add(const void* a, const void* b, void* y, long n, bool relu);
void relu_mask(const void* dy, const void* y, void* dx, long n);
void adam(float* p, const float* g, float* m, float* v, void* shadow, long n, float lr, float b1, float b2, float eps,
          float bc1, float bc2, float wd, bool decoupled);
void sgd(float* p, const float* g, float* vel, void* shadow, long n, float lr, float momentum);
// device-resident Adam step scalars hyper = {lr, bc1, bc2, t} (a captured step replays with the
// current values): t += 1 and the bias corrections on the device, then the fused update reading them
void adam_hyper_step(float* hyper, float b1, float b2);
void adam_dev(float* p, const float* g, float* m, float* v, void* shadow, long n, float b1, float b2, float eps,
              float wd, bool decoupled, const float* hyper);
// {loss (fp32), -, correct (int32)} of the last fused loss launch (read after a graph replay)
const void* loss_device();
}  // namespace gpu_ops

}  // namespace dcnn
