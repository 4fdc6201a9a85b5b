// CPU backend of the C++ host API: fp32 NCHW on the native CPU kernels (csrc/native/cpu_ops.cpp,
// cpu_gemm.cpp — the same routines the Python CPU path runs).
#include "../native/cpu_kernels.h"
#include "dcnn/ops.hpp"

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

void adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps, float bc1,
          float bc2, float wd, bool decoupled) {
  C::adam_step(p, g, m, v, n, lr, b1, b2, eps, bc1, bc2, wd, decoupled ? 1 : 0);
}

void sgd(float* p, const float* g, float* vel, long n, float lr, float momentum) {
  C::sgd_step(p, g, vel, n, lr, momentum);
}

}  // namespace cpu_ops
}  // namespace dcnn
