// CPU backend of the C++ host API: fp32 NCHW on the native CPU kernels (csrc/native/cpu_ops.cpp,
// cpu_gemm.cpp — the same routines the Python CPU path runs).
#include "../native/cpu_kernels.h"
#include "dcnn/ops.hpp"

#include <stdexcept>

namespace dcnn {
namespace cpu_ops {
namespace C = dcnn_native::cpu;

void conv_fwd(const float* x, const float* w, const float* b, float* y, const ConvShape& s) {
  C::conv2d_fwd(x, w, b, y, s.N, s.C, s.H, s.W, s.Co, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW);
}

void conv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, const ConvShape& s) {
  C::conv2d_bwd(x, w, dy, dx, dw, db, s.N, s.C, s.H, s.W, s.Co, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW);
}

void dense_fwd(const float* x, const float* w, const float* b, float* y, long N, long In, long Out) {
  C::dense_fwd(x, w, b, y, N, In, Out);
}

void dense_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, long N, long In,
               long Out) {
  C::dense_bwd(x, w, dy, dx, dw, db, N, In, Out);
}

void bn_fwd(const float* x, float* y, long N, long Cc, long HW, const float* g, const float* b, float eps, bool train,
            float* rmean, float* rvar, float momentum, float* smean, float* sistd) {
  C::batchnorm_fwd<float>(x, y, N, Cc, HW, g, b, eps, train ? 1 : 0, rmean, rvar, momentum, smean, sistd, 0, nullptr);
}

void bn_bwd(const float* x, const float* dy, const float* mean, const float* istd, const float* g, float* dx,
            float* dg, float* db, long N, long Cc, long HW, bool train) {
  C::batchnorm_bwd<float>(x, dy, nullptr, mean, istd, g, dx, dg, db, nullptr, N, Cc, HW, train ? 1 : 0);
}

void maxpool_fwd(const float* x, float* y, int32_t* idx, const PoolShape& p) {
  C::maxpool_fwd(x, y, idx, (long)p.N * p.C, p.H, p.W, p.KH, p.KW, p.SH, p.SW, p.PH, p.PW);
}

void maxpool_bwd(const float* dy, const int32_t* idx, float* dx, const PoolShape& p) {
  C::maxpool_bwd(dy, idx, dx, (long)p.N * p.C, p.H, p.W, p.OH, p.OW);
}

void avgpool_fwd(const float* x, float* y, const PoolShape& p) {
  C::avgpool_fwd(x, y, (long)p.N * p.C, p.H, p.W, p.KH, p.KW, p.SH, p.SW, p.PH, p.PW);
}

void avgpool_bwd(const float* dy, float* dx, const PoolShape& p) {
  C::avgpool_bwd(dy, dx, (long)p.N * p.C, p.H, p.W, p.KH, p.KW, p.SH, p.SW, p.PH, p.PW);
}

// the CPU kernels number activations 0 linear, 1 relu, 2 leaky, 3 elu, 4 sigmoid, 5 tanh
static int cpu_act(int kind) {
  static const int map[] = {1, 2, 3, 4, 5, 0};
  return map[kind];
}

void act_fwd(int kind, const float* x, float* y, long n, float alpha) { C::act_fwd(cpu_act(kind), x, y, n, alpha); }

void act_bwd(int kind, const float* x, const float* dy, float* dx, long n, float alpha) {
  C::act_bwd(cpu_act(kind), x, dy, dx, n, alpha);
}

double softmax_ce(const float* pred, const int64_t* labels, float* grad, long N, long Cc, long* correct) {
  return C::loss_fused(1, pred, (const float*)nullptr, labels, grad, N, Cc, 1e-15, correct);
}

double loss(int kind, const float* pred, const float* target, const int64_t* labels, float* grad, long N, long Cc,
            float param, long* correct) {
  // the CPU kernels number the losses 0 ce, 1 softmax ce (= log-softmax ce), 2 mse, 3 mae, 4 huber
  static const int map[] = {0, 1, 1, 2, 3, 4};
  if (kind < 0 || kind > 5) throw std::invalid_argument("loss: unknown kind");
  return C::loss_fused(map[kind], pred, target, labels, grad, N, Cc, param, correct);
}

void groupnorm_fwd(const float* x, float* y, long N, long Cc, long HW, long G, const float* g, const float* b, float eps,
                   float* smean, float* sistd) {
  C::groupnorm_fwd<float>(x, y, N, Cc, HW, G, g, b, eps, smean, sistd);
}

void groupnorm_bwd(const float* x, const float* dy, const float* mean, const float* istd, const float* g, float* dx,
                   float* dg, float* db, long N, long Cc, long HW, long G) {
  C::groupnorm_bwd<float>(x, dy, mean, istd, g, dx, dg, db, N, Cc, HW, G);
}

void softmax_fwd(const float* x, float* y, long N, long Cc, long HW) { C::softmax_channels<float>(x, y, N, Cc, HW); }
void softmax_bwd(const float* y, const float* dy, float* dx, long N, long Cc, long HW) {
  C::softmax_channels_bwd<float>(y, dy, dx, N, Cc, HW);
}

void dropout(const float* x, float* y, long n, float p, uint64_t seed) {
  // counter-based mask (splitmix64 of seed ^ index): the backward call regenerates it exactly
  const float scale = 1.f / (1.f - p);
  for (long i = 0; i < n; ++i) {
    uint64_t z = seed + 0x9e3779b97f4a7c15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    const float u = (float)((z >> 40) * (1.0 / 16777216.0));
    y[i] = u >= p ? x[i] * scale : 0.f;
  }
}

void add(const float* a, const float* b, float* y, long n, bool relu) {
  for (long i = 0; i < n; ++i) {
    const float v = a[i] + b[i];
    y[i] = relu && v < 0.f ? 0.f : v;
  }
}

void relu_mask(const float* dy, const float* y, float* dx, long n) {
  for (long i = 0; i < n; ++i) dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

void adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps, float bc1,
          float bc2, float wd, bool decoupled) {
  C::adam_step(p, g, m, v, n, lr, b1, b2, eps, bc1, bc2, wd, decoupled ? 1 : 0);
}

void sgd(float* p, const float* g, float* vel, long n, float lr, float momentum) {
  C::sgd_step(p, g, vel, n, lr, momentum);
}

}  // namespace cpu_ops
}  // namespace dcnn
