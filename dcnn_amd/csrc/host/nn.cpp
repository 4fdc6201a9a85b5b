// Layers, Sequential, loss, optimizers and the training loop of the C++ host API (dcnn/nn.hpp).
#include "dcnn/nn.hpp"

#include "../kernels/fusion_plan.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

namespace dcnn {

namespace {
// splitmix64 stream: deterministic initialisation independent of the platform RNG
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  float uniform() { return (float)((next() >> 40) * (1.0 / 16777216.0)); }  // [0, 1)
  float normal() {
    const float u1 = std::max(uniform(), 1e-7f), u2 = uniform();
    return std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
  }
};

std::vector<float> uniform_init(size_t n, float bound, uint64_t seed) {
  Rng r(seed);
  std::vector<float> v(n);
  for (auto& x : v) x = (2.f * r.uniform() - 1.f) * bound;
  return v;
}

// activations: CPU fp32 NCHW, GPU bf16 NHWC
Tensor act_empty(const std::vector<int64_t>& shape, Device dev) {
  return dev.is_gpu() ? Tensor::empty(shape, DType::BF16, dev, Layout::NHWC) : Tensor::empty(shape, DType::F32, dev);
}

void check_act(const Tensor& x, Device dev, const char* who) {
  if (x.device() != dev) throw std::runtime_error(std::string(who) + ": input on " + x.device().str() +
                                                  ", layer on " + dev.str());
  if (x.rank() != 4) throw std::runtime_error(std::string(who) + ": expected an (N, C, H, W) tensor");
}

constexpr int ACT_SOFTMAX = 100;  // (channel softmax: its own kernels, not an elementwise one)

int act_code(const std::string& k) {
  if (k == "softmax") return ACT_SOFTMAX;
  if (k == "relu") return ACT_RELU;
  if (k == "leaky_relu") return ACT_LEAKY_RELU;
  if (k == "elu") return ACT_ELU;
  if (k == "sigmoid") return ACT_SIGMOID;
  if (k == "tanh") return ACT_TANH;
  if (k == "linear") return ACT_LINEAR;
  throw std::invalid_argument("unknown activation '" + k + "'");
}
}  // namespace

// ------------------------------------------------------------------ Layer
Param& Layer::add_param(const std::string& n, const std::vector<int64_t>& shape, Layout phys,
                        const std::vector<float>& init) {
  Param p;
  p.name = n;
  p.shape = shape;
  p.layout = phys;
  p.value = Tensor::from_host(init, shape, dev_, DType::F32, phys);
  p.grad = Tensor::zeros(shape, DType::F32, dev_, phys);
  if (dev_.is_gpu()) {
    p.shadow = Tensor::empty(shape, DType::BF16, dev_, phys);
    gpu_ops::cast_bf16(p.value.ptr<float>(), p.shadow.data(), p.value.numel());
  }
  params_.push_back(std::move(p));
  return params_.back();
}

void Layer::sync_shadow() {
  for (auto& p : params_)
    if (p.shadow.defined()) gpu_ops::cast_bf16(p.value.ptr<float>(), p.shadow.data(), p.value.numel());
}

// ------------------------------------------------------------------ Conv2D
Conv2D::Conv2D(int in_ch, int out_ch, int kh, int kw, int sh, int sw, int ph, int pw, bool bias, std::string name)
    : Layer(std::move(name)), ci_(in_ch), co_(out_ch), kh_(kh), kw_(kw), sh_(sh), sw_(sw), ph_(ph), pw_(pw),
      bias_(bias) {}

json::Value Conv2D::parameters_config() const {
  json::Value p = json::Value::object();
  p["in_channels"] = ci_;
  p["out_channels"] = co_;
  p["kernel_h"] = kh_;
  p["kernel_w"] = kw_;
  p["stride_h"] = sh_;
  p["stride_w"] = sw_;
  p["pad_h"] = ph_;
  p["pad_w"] = pw_;
  p["use_bias"] = bias_;
  p["optimized"] = "mfma";
  return p;
}

ConvShape Conv2D::shape_for(const std::vector<int64_t>& in) const {
  ConvShape s{};
  s.N = (int)in[0];
  s.C = (int)in[1];
  s.H = (int)in[2];
  s.W = (int)in[3];
  s.Co = co_;
  s.KH = kh_;
  s.KW = kw_;
  s.SH = sh_;
  s.SW = sw_;
  s.PH = ph_;
  s.PW = pw_;
  s.OH = (s.H + 2 * ph_ - kh_) / sh_ + 1;
  s.OW = (s.W + 2 * pw_ - kw_) / sw_ + 1;
  if (s.C != ci_) throw std::runtime_error(name_ + ": input has " + std::to_string(s.C) + " channels, expected " +
                                           std::to_string(ci_));
  return s;
}

std::vector<int64_t> Conv2D::output_shape(const std::vector<int64_t>& in) const {
  const ConvShape s = shape_for(in);
  return {in[0], co_, s.OH, s.OW};
}

void Conv2D::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  (void)in;
  dev_ = dev;
  params_.clear();
  const float bound = 1.f / std::sqrt((float)(ci_ * kh_ * kw_));
  // GPU: physical [Co][KH][KW][Ci] (the GEMM B operand); CPU: NCHW
  const Layout wl = dev.is_gpu() ? Layout::NHWC : Layout::NCHW;
  add_param("weights", {co_, ci_, kh_, kw_}, wl, uniform_init((size_t)co_ * ci_ * kh_ * kw_, bound, seed));
  if (bias_) add_param("bias", {co_, 1, 1, 1}, Layout::NCHW, uniform_init((size_t)co_, bound, seed + 1));
}

double Conv2D::flops(const std::vector<int64_t>& in) const {
  const ConvShape s = shape_for(in);
  const double out = (double)s.N * s.OH * s.OW, k = (double)ci_ * kh_ * kw_;
  return 6.0 * co_ * k * out + (bias_ ? 2.0 * co_ * out : 0.0);  // forward 2, backward 4 per MAC
}

bool Conv2D::takes_raw_input(const std::vector<int64_t>& in) const {
  return dev_.is_gpu() && in.size() == 4 && in[1] == ci_ && gpu_ops::stem_ok(shape_for(in));
}

Tensor Conv2D::forward(const Tensor& x, bool training) {
  Tensor& x_ = mbc().a;
  check_act(x, dev_, "conv2d");
  const ConvShape s = shape_for(x.shape());
  Tensor y = act_empty({s.N, s.Co, s.OH, s.OW}, dev_);
  const float* b = bias_ ? params_[1].value.ptr<float>() : nullptr;
  if (dev_.is_gpu() && x.dtype() == DType::F32) {
    // the network input, fp32 NCHW, on the RGB stem kernel (Sequential::input_activation)
    if (x.layout() != Layout::NCHW || !gpu_ops::stem_ok(s)) throw std::runtime_error(name_ + ": fp32 input");
    int rows = 0;
    const float* st = gpu_ops::stem_fwd(x.ptr<float>(), params_[0].shadow.data(), b, y.data(), s,
                                        stats_to_ && training ? &rows : nullptr);
    if (stats_to_ && training) stats_to_->offer_stats(y.data(), st, rows);
    x_ = x;
    return y;
  }
  if (dev_.is_gpu()) {
    int rows = 0;
    const float* st = gpu_ops::conv_fwd(x.data(), params_[0].shadow.data(), b, y.data(), s,
                                        stats_to_ && training ? &rows : nullptr);
    if (stats_to_ && training) stats_to_->offer_stats(y.data(), st, rows);
  } else
    cpu_ops::conv_fwd(x.ptr<float>(), params_[0].value.ptr<float>(), b, y.ptr<float>(), s);
  x_ = x;
  return y;
}

bool Conv2D::ran_stem() const {
  const Tensor& x_ = const_cast<Conv2D*>(this)->mbc().a;
  return dev_.is_gpu() && x_.defined() && x_.dtype() == DType::F32;
}

void Conv2D::backward_stem_bn(const Tensor& dy, const gpu_ops::StemBn& bn) {
  const Tensor& x_ = mbc().a;
  const ConvShape s = shape_for(x_.shape());
  gpu_ops::stem_wgrad_bn(dy.data(), x_.ptr<float>(), params_[0].grad.ptr<float>(),
                         bias_ ? params_[1].grad.ptr<float>() : nullptr, s, bn);
}

Tensor Conv2D::backward(const Tensor& dy) {
  const Tensor& x_ = mbc().a;
  const ConvShape s = shape_for(x_.shape());
  float* gb = bias_ ? params_[1].grad.ptr<float>() : nullptr;
  if (dev_.is_gpu() && x_.dtype() == DType::F32) {  // stem: the input needs no gradient
    gpu_ops::stem_wgrad(dy.data(), x_.ptr<float>(), params_[0].grad.ptr<float>(), gb, s);
    return Tensor();
  }
  if (dev_.is_gpu()) {
    gpu_ops::conv_wgrad(dy.data(), x_.data(), params_[0].grad.ptr<float>(), gb, s);
    if (!input_grad_) return Tensor();
    Tensor dx = act_empty(x_.shape(), dev_);
    bool tr = false;
    const void* w = dgrad_operand(tr);
    if (bnb_from_ != nullptr) {
      const gpu_ops::BnbOperands ops = bnb_from_->bnb_operands(mb_);
      int rows = 0;
      const float* st = gpu_ops::conv_dgrad(dy.data(), w, dx.data(), s, nullptr, tr, &ops, &rows);
      if (rows > 0) bnb_from_->offer_bwd_stats(dx.data(), st, rows);
      return dx;
    }
    gpu_ops::conv_dgrad(dy.data(), w, dx.data(), s, nullptr, tr);
    return dx;
  }
  Tensor dx = act_empty(x_.shape(), dev_);
  {
    cpu_ops::conv_bwd(x_.ptr<float>(), params_[0].value.ptr<float>(), dy.ptr<float>(), dx.ptr<float>(),
                      params_[0].grad.ptr<float>(), gb, s);
  }
  return dx;
}

Tensor Conv2D::backward_residual(const Tensor& dy, const Tensor& residual) {
  const Tensor& x_ = mbc().a;
  if (!dev_.is_gpu() || x_.dtype() == DType::F32 || residual.shape() != x_.shape())
    throw std::runtime_error(name_ + ": backward_residual is a GPU fusion");
  const ConvShape s = shape_for(x_.shape());
  float* gb = bias_ ? params_[1].grad.ptr<float>() : nullptr;
  gpu_ops::conv_wgrad(dy.data(), x_.data(), params_[0].grad.ptr<float>(), gb, s);
  Tensor dx = act_empty(x_.shape(), dev_);
  bool tr = false;
  const void* w = dgrad_operand(tr);
  if (bnb_block_from_ != nullptr) {
    const gpu_ops::BnbOperands ops = bnb_block_from_->bnb_operands(mb_);
    int rows = 0;
    const float* st = gpu_ops::conv_dgrad(dy.data(), w, dx.data(), s, residual.data(), tr, &ops, &rows);
    if (rows > 0) bnb_block_from_->offer_bwd_stats(dx.data(), st, rows);
    return dx;
  }
  gpu_ops::conv_dgrad(dy.data(), w, dx.data(), s, residual.data(), tr);
  return dx;
}

gpu_ops::BnbOperands BatchNorm::bnb_operands(int mb) {
  set_micro_batch(mb);
  MbCache& mc = mbc();
  gpu_ops::BnbOperands o{mc.d.defined() ? mc.d.data() : nullptr, mc.a.data(), mc.b.ptr<float>(), mc.c.ptr<float>()};
  if (mc.d.defined() && mc.flag) {  // (mc.flag: mc.d is a plain BN + ReLU output, forward_impl)
    o.gamma = affine_ ? params_[0].value.ptr<float>() : nullptr;
    o.beta = affine_ ? params_[1].value.ptr<float>() : nullptr;
    o.mask_from_x = true;
  }
  return o;
}

bool Conv2D::make_transposed_operand(std::vector<int64_t>& row, long& tiles) {
  if (!dev_.is_gpu() || ci_ % 8 || co_ % 8 || params_.empty()) return false;
  wt_ = Tensor::empty({ci_, kh_, kw_, co_}, DType::BF16, dev_);
  row = {(int64_t)(uintptr_t)params_[0].shadow.data(), (int64_t)(uintptr_t)wt_.data(), co_, kh_ * kw_, ci_};
  tiles = (long)kh_ * kw_ * ((co_ + 63) / 64) * ((ci_ + 63) / 64);
  return true;
}

void Conv2D::sync_shadow() {
  Layer::sync_shadow();
  if (wt_.defined()) gpu_ops::weight_transpose(params_[0].shadow.data(), wt_.data(), co_, kh_ * kw_, ci_);
}

const void* Conv2D::dgrad_operand(bool& transposed) const {
  const ParamArena* a = params_[0].arena.get();
  transposed = wt_.defined() && a != nullptr && a->wt_valid;
  return transposed ? wt_.data() : params_[0].shadow.data();
}

void ParamArena::refresh_transposes() {
  if (n_wt == 0) return;
  gpu_ops::multi_weight_transpose(wt_table.ptr<int64_t>(), n_wt, wt_tiles);
  wt_valid = true;
}

// ------------------------------------------------------------------ Dense
Dense::Dense(int in_features, int out_features, bool bias, std::string name)
    : Layer(std::move(name)), in_(in_features), out_(out_features), bias_(bias) {}

json::Value Dense::parameters_config() const {
  json::Value p = json::Value::object();
  p["input_features"] = in_;
  p["output_features"] = out_;
  p["use_bias"] = bias_;
  p["optimized"] = "mfma";
  return p;
}

std::vector<int64_t> Dense::output_shape(const std::vector<int64_t>& in) const {
  if (in[1] * in[2] * in[3] != in_)
    throw std::runtime_error(name_ + ": " + std::to_string(in[1] * in[2] * in[3]) + " input features, expected " +
                             std::to_string(in_));
  return {in[0], out_, 1, 1};
}

void Dense::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  (void)in;
  dev_ = dev;
  params_.clear();
  const float bound = 1.f / std::sqrt((float)in_);
  add_param("weights", {out_, in_, 1, 1}, Layout::NCHW, uniform_init((size_t)out_ * in_, bound, seed));
  if (bias_) add_param("bias", {out_, 1, 1, 1}, Layout::NCHW, uniform_init((size_t)out_, bound, seed + 1));
}

Tensor Dense::forward(const Tensor& x, bool training) {
  (void)training;
  Tensor& x_ = mbc().a;
  check_act(x, dev_, "dense");
  const int N = (int)x.dim(0);
  output_shape(x.shape());
  Tensor y = act_empty({N, out_, 1, 1}, dev_);
  const float* b = bias_ ? params_[1].value.ptr<float>() : nullptr;
  if (dev_.is_gpu())
    gpu_ops::dense_fwd(x.data(), params_[0].shadow.data(), b, y.data(), N, in_, out_);
  else
    cpu_ops::dense_fwd(x.ptr<float>(), params_[0].value.ptr<float>(), b, y.ptr<float>(), N, in_, out_);
  x_ = x;
  return y;
}

Tensor Dense::backward(const Tensor& dy) {
  const Tensor& x_ = mbc().a;
  const int N = (int)x_.dim(0);
  float* gb = bias_ ? params_[1].grad.ptr<float>() : nullptr;
  if (dev_.is_gpu()) {
    gpu_ops::dense_wgrad(dy.data(), x_.data(), params_[0].grad.ptr<float>(), gb, N, in_, out_);
    if (!input_grad_) return Tensor();
    Tensor dx = act_empty(x_.shape(), dev_);
    gpu_ops::dense_dgrad(dy.data(), params_[0].shadow.data(), dx.data(), N, in_, out_);
    return dx;
  }
  Tensor dx = act_empty(x_.shape(), dev_);
  {
    cpu_ops::dense_bwd(x_.ptr<float>(), params_[0].value.ptr<float>(), dy.ptr<float>(), dx.ptr<float>(),
                       params_[0].grad.ptr<float>(), gb, N, in_, out_);
  }
  return dx;
}

// ------------------------------------------------------------------ BatchNorm
BatchNorm::BatchNorm(int num_features, float eps, float momentum, bool affine, std::string name)
    : Layer(std::move(name)), c_(num_features), eps_(eps), momentum_(momentum), affine_(affine) {}

json::Value BatchNorm::parameters_config() const {
  json::Value p = json::Value::object();
  p["num_features"] = c_;
  p["epsilon"] = (double)eps_;
  p["momentum"] = (double)momentum_;
  p["affine"] = affine_;
  return p;
}

void BatchNorm::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  (void)in;
  (void)seed;
  dev_ = dev;
  params_.clear();
  if (affine_) {
    add_param("gamma", {c_, 1, 1, 1}, Layout::NCHW, std::vector<float>((size_t)c_, 1.f));
    add_param("beta", {c_, 1, 1, 1}, Layout::NCHW, std::vector<float>((size_t)c_, 0.f));
  }
  running_mean = Tensor::zeros({c_}, DType::F32, dev);
  running_var = Tensor::from_host(std::vector<float>((size_t)c_, 1.f), {c_}, dev);
  caches_.clear();
}

Tensor BatchNorm::forward(const Tensor& x, bool training) { return forward_impl(x, training, nullptr, fused_relu_); }

Tensor BatchNorm::forward_residual(const Tensor& x, const Tensor& residual, bool relu, bool training) {
  if (!dev_.is_gpu()) throw std::runtime_error(name_ + ": forward_residual is a GPU fusion");
  if (residual.shape() != x.shape()) throw std::runtime_error(name_ + ": residual shape mismatch");
  return forward_impl(x, training, &residual, relu);
}

Tensor BatchNorm::forward_impl(const Tensor& x, bool training, const Tensor* residual, bool relu) {
  check_act(x, dev_, "batchnorm");
  MbCache& mc = mbc();
  Tensor& x_ = mc.a;
  Tensor& mean_ = mc.b;
  Tensor& istd_ = mc.c;
  mean_.ensure({c_}, DType::F32, dev_);
  istd_.ensure({c_}, DType::F32, dev_);
  if (x.dim(1) != c_) throw std::runtime_error(name_ + ": channel count mismatch");
  train_ = training;
  const long N = x.dim(0), HW = x.dim(2) * x.dim(3);
  Tensor y = act_empty(x.shape(), dev_);
  const float* g = affine_ ? params_[0].value.ptr<float>() : nullptr;
  const float* b = affine_ ? params_[1].value.ptr<float>() : nullptr;
  const void* res = residual ? residual->data() : nullptr;
  const bool slab = dev_.is_gpu() && training && pending_x_ == x.data() && pending_slab_ && pending_rows_ > 0;
  if (fused_pool_ != nullptr) {
    fused_pool_->set_micro_batch(mb_);  // (its own forward sets it only after this one)
    const PoolShape p = fused_pool_->shape_for(x.shape());
    if (dev_.is_gpu() && training && relu && residual == nullptr && gpu_ops::bn_relu_maxpool_ok(p)) {
      // BatchNorm + ReLU + max-pool in one pass: the full-resolution output is never stored, the
      // pool layer passes this result through (its backward masks with the pooled value)
      Tensor yp = act_empty({p.N, p.C, p.OH, p.OW}, dev_);
      uint8_t* idx = fused_pool_->accept_prepooled(yp, x.shape());
      gpu_ops::bn_relu_maxpool(x.data(), yp.data(), idx, p, slab ? pending_slab_ : nullptr, slab ? pending_rows_ : 0,
                               g, b, eps_, running_mean.ptr<float>(), running_var.ptr<float>(), momentum_,
                               mean_.ptr<float>(), istd_.ptr<float>());
      mc.d = Tensor();
      mc.flag = false;
      pending_x_ = nullptr;
      pending_slab_ = nullptr;
      pending_rows_ = 0;
      x_ = x;
      return yp;
    }
    fused_pool_->clear_prepooled();
  }
  if (slab) {  // statistics from the producing conv's epilogue
    gpu_ops::bn_fwd_slab(x.data(), y.data(), N * HW, c_, pending_slab_, pending_rows_, g, b, eps_,
                         running_mean.ptr<float>(), running_var.ptr<float>(), momentum_, mean_.ptr<float>(),
                         istd_.ptr<float>(), relu, res);
    mc.d = relu ? y : Tensor();  // (the ReLU mask of the backward)
    mc.flag = relu && res == nullptr && training;  // (the mask is a function of x: bnb_operands)
  } else if (dev_.is_gpu()) {
    gpu_ops::bn_fwd(x.data(), y.data(), N * HW, c_, g, b, eps_, training, running_mean.ptr<float>(),
                    running_var.ptr<float>(), momentum_, mean_.ptr<float>(), istd_.ptr<float>(), relu, res);
    mc.d = relu ? y : Tensor();
    mc.flag = relu && res == nullptr && training;
  } else {
    cpu_ops::bn_fwd(x.ptr<float>(), y.ptr<float>(), N, c_, HW, g, b, eps_, training, running_mean.ptr<float>(),
                    running_var.ptr<float>(), momentum_, mean_.ptr<float>(), istd_.ptr<float>());
  }
  pending_x_ = nullptr;
  pending_slab_ = nullptr;
  pending_rows_ = 0;
  x_ = x;
  return y;
}

void BatchNorm::forward_deferred(const Tensor& x, bool training) {
  check_act(x, dev_, "batchnorm");
  if (!dev_.is_gpu()) throw std::runtime_error(name_ + ": forward_deferred is a GPU fusion");
  if (x.dim(1) != c_) throw std::runtime_error(name_ + ": channel count mismatch");
  MbCache& mc = mbc();
  mc.a = x;
  mc.b.ensure({c_}, DType::F32, dev_);
  mc.c.ensure({c_}, DType::F32, dev_);
  mc.d = Tensor();
  mc.flag = false;
  train_ = training;
  deferred_raw_ = gpu_ops::BnRaw{nullptr, 0};
  if (training) {
    const bool slab = pending_x_ == x.data() && pending_slab_ && pending_rows_ > 0;
    deferred_raw_ = gpu_ops::bn_stats_raw(x.data(), x.dim(0) * x.dim(2) * x.dim(3), c_, slab ? pending_slab_ : nullptr,
                                          slab ? pending_rows_ : 0);
  }
  pending_x_ = nullptr;
  pending_slab_ = nullptr;
  pending_rows_ = 0;
}

// the deferred BatchNorm's own output (when the consumer cannot pair it)
Tensor BatchNorm::apply_deferred(bool training) {
  MbCache& mc = mbc();
  const Tensor& x = mc.a;
  const long R = x.dim(0) * x.dim(2) * x.dim(3);
  Tensor y = act_empty(x.shape(), dev_);
  const float* g = affine_ ? params_[0].value.ptr<float>() : nullptr;
  const float* b = affine_ ? params_[1].value.ptr<float>() : nullptr;
  if (training)
    gpu_ops::bn_fwd_slab(x.data(), y.data(), R, c_, deferred_raw_.slab, deferred_raw_.rows, g, b, eps_,
                         running_mean.ptr<float>(), running_var.ptr<float>(), momentum_, mc.b.ptr<float>(),
                         mc.c.ptr<float>(), false);
  else
    gpu_ops::bn_fwd(x.data(), y.data(), R, c_, g, b, eps_, false, running_mean.ptr<float>(), running_var.ptr<float>(),
                    momentum_, mc.b.ptr<float>(), mc.c.ptr<float>());
  return y;
}

Tensor BatchNorm::forward_dual(const Tensor& x, BatchNorm& o, bool relu, bool training) {
  check_act(x, dev_, "batchnorm");
  if (x.dim(1) != c_) throw std::runtime_error(name_ + ": channel count mismatch");
  MbCache& oc = o.mbc();
  const long R = x.dim(0) * x.dim(2) * x.dim(3);
  if (oc.a.shape() != x.shape() || o.c_ != c_ || !gpu_ops::bn_dual_ok(R, c_)) {
    const Tensor ys = o.apply_deferred(training);
    return forward_impl(x, training, &ys, relu);
  }
  MbCache& mc = mbc();
  mc.b.ensure({c_}, DType::F32, dev_);
  mc.c.ensure({c_}, DType::F32, dev_);
  train_ = training;
  gpu_ops::BnRaw raw{nullptr, 0};
  if (training) {
    const bool slab = pending_x_ == x.data() && pending_slab_ && pending_rows_ > 0;
    raw = gpu_ops::bn_stats_raw(x.data(), R, c_, slab ? pending_slab_ : nullptr, slab ? pending_rows_ : 0);
  }
  auto side = [](BatchNorm& l, MbCache& c, const gpu_ops::BnRaw& r) {
    return gpu_ops::BnFwdSide{c.a.data(),
                              r,
                              l.affine_ ? l.params_[0].value.ptr<float>() : nullptr,
                              l.affine_ ? l.params_[1].value.ptr<float>() : nullptr,
                              l.eps_,
                              l.running_mean.ptr<float>(),
                              l.running_var.ptr<float>(),
                              l.momentum_,
                              c.b.ptr<float>(),
                              c.c.ptr<float>()};
  };
  mc.a = x;
  Tensor y = act_empty(x.shape(), dev_);
  gpu_ops::bn_fwd_dual(side(*this, mc, raw), side(o, oc, o.deferred_raw_), y.data(), R, c_, relu, training);
  mc.d = relu ? y : Tensor();
  mc.flag = false;
  pending_x_ = nullptr;
  pending_slab_ = nullptr;
  pending_rows_ = 0;
  o.deferred_raw_ = gpu_ops::BnRaw{nullptr, 0};
  return y;
}

bool BatchNorm::backward_dual(const Tensor& dy, BatchNorm& o, Tensor& dx, Tensor& dx_o) {
  MbCache& mc = mbc();
  MbCache& oc = o.mbc();
  const Tensor& x_ = mc.a;
  if (!dev_.is_gpu() || bwd_dy_ != dy.data() || bwd_slab_ == nullptr || bwd_rows_ <= 0 || !train_ || !o.train_ ||
      oc.a.shape() != x_.shape() || o.c_ != c_)
    return false;
  const long R = x_.dim(0) * x_.dim(2) * x_.dim(3);
  if (!gpu_ops::bn_dual_ok(R, c_)) return false;
  dx = act_empty(x_.shape(), dev_);
  dx_o = act_empty(oc.a.shape(), dev_);
  auto side = [](BatchNorm& l, MbCache& c, Tensor& d) {
    return gpu_ops::BnBwdSides{c.a.data(),
                               d.data(),
                               c.b.ptr<float>(),
                               c.c.ptr<float>(),
                               l.affine_ ? l.params_[0].value.ptr<float>() : nullptr,
                               l.affine_ ? l.params_[0].grad.ptr<float>() : nullptr,
                               l.affine_ ? l.params_[1].grad.ptr<float>() : nullptr};
  };
  gpu_ops::bn_bwd_dual(dy.data(), side(*this, mc, dx), bwd_slab_, bwd_rows_, side(o, oc, dx_o), R, c_);
  bwd_dy_ = nullptr;
  bwd_slab_ = nullptr;
  bwd_rows_ = 0;
  return true;
}

Tensor BatchNorm::backward_residual(const Tensor& dy, Tensor* branch) {
  MbCache& mc = mbc();
  const Tensor& x_ = mc.a;
  const long N = x_.dim(0), HW = x_.dim(2) * x_.dim(3);
  Tensor dx = act_empty(x_.shape(), dev_);
  const float* g = affine_ ? params_[0].value.ptr<float>() : nullptr;
  float* dg = affine_ ? params_[0].grad.ptr<float>() : nullptr;
  float* db = affine_ ? params_[1].grad.ptr<float>() : nullptr;
  if (bwd_dy_ == dy.data() && bwd_slab_ != nullptr && bwd_rows_ > 0) {
    // dy already masked and its statistics computed by the next block's head-conv dgrad
    *branch = dy;
    gpu_ops::bn_bwd_slab(dy.data(), x_.data(), dx.data(), N * HW, c_, mc.b.ptr<float>(), mc.c.ptr<float>(), g, dg, db,
                         train_, bwd_slab_, bwd_rows_);
    bwd_dy_ = nullptr;
    bwd_slab_ = nullptr;
    bwd_rows_ = 0;
  } else if (mc.d.defined()) {
    *branch = act_empty(dy.shape(), dev_);
    gpu_ops::bn_bwd(dy.data(), x_.data(), dx.data(), N * HW, c_, mc.b.ptr<float>(), mc.c.ptr<float>(), g, dg, db,
                    train_, mc.d.data(), branch->data());
  } else {
    *branch = dy;
    gpu_ops::bn_bwd(dy.data(), x_.data(), dx.data(), N * HW, c_, mc.b.ptr<float>(), mc.c.ptr<float>(), g, dg, db,
                    train_);
  }
  return dx;
}

bool BatchNorm::backward_into_stem(const Tensor& dy, Conv2D& stem) {
  MbCache& mc = mbc();
  if (!dev_.is_gpu() || !train_ || bwd_dy_ != dy.data() || bwd_slab_ == nullptr || bwd_rows_ <= 0 ||
      !stem.ran_stem() || mc.a.dtype() != DType::BF16)
    return false;
  gpu_ops::StemBn bn{mc.a.data(),
                     mc.b.ptr<float>(),
                     mc.c.ptr<float>(),
                     affine_ ? params_[0].value.ptr<float>() : nullptr,
                     affine_ ? params_[0].grad.ptr<float>() : nullptr,
                     affine_ ? params_[1].grad.ptr<float>() : nullptr,
                     bwd_slab_,
                     bwd_rows_,
                     train_};
  stem.backward_stem_bn(dy, bn);
  bwd_dy_ = nullptr;
  bwd_slab_ = nullptr;
  bwd_rows_ = 0;
  return true;
}

Tensor BatchNorm::backward(const Tensor& dy) {
  MbCache& mc = mbc();
  const Tensor& x_ = mc.a;
  Tensor& mean_ = mc.b;
  Tensor& istd_ = mc.c;
  const long N = x_.dim(0), HW = x_.dim(2) * x_.dim(3);
  Tensor dx = act_empty(x_.shape(), dev_);
  const float* g = affine_ ? params_[0].value.ptr<float>() : nullptr;
  float* dg = affine_ ? params_[0].grad.ptr<float>() : nullptr;
  float* db = affine_ ? params_[1].grad.ptr<float>() : nullptr;
  if (dev_.is_gpu() && bwd_dy_ == dy.data() && bwd_slab_ != nullptr && bwd_rows_ > 0) {
    // statistics (and the ReLU mask) from the consuming conv's data-gradient epilogue
    gpu_ops::bn_bwd_slab(dy.data(), x_.data(), dx.data(), N * HW, c_, mean_.ptr<float>(), istd_.ptr<float>(), g, dg,
                         db, train_, bwd_slab_, bwd_rows_);
    bwd_dy_ = nullptr;
    bwd_slab_ = nullptr;
    bwd_rows_ = 0;
  } else if (dev_.is_gpu())
    gpu_ops::bn_bwd(dy.data(), x_.data(), dx.data(), N * HW, c_, mean_.ptr<float>(), istd_.ptr<float>(), g, dg, db,
                    train_, mc.d.defined() ? mc.d.data() : nullptr);
  else
    cpu_ops::bn_bwd(x_.ptr<float>(), dy.ptr<float>(), mean_.ptr<float>(), istd_.ptr<float>(), g, dx.ptr<float>(), dg,
                    db, N, c_, HW, train_);
  return dx;
}

// ------------------------------------------------------------------ Activation
Activation::Activation(std::string kind, std::string name)
    : Layer(std::move(name)), kind_(std::move(kind)), code_(act_code(kind_)) {}

json::Value Activation::parameters_config() const {
  json::Value p = json::Value::object();
  p["activation"] = kind_;
  return p;
}

static float act_alpha(int code) { return code == ACT_ELU ? 1.0f : 0.01f; }

bool Activation::is_relu() const { return code_ == ACT_RELU; }

// a layer's kind for the shared fusion planner (csrc/kernels/fusion_plan.h)
static int fuse_kind(const Layer* l) {
  if (dynamic_cast<const Conv2D*>(l)) return FK_CONV;
  if (dynamic_cast<const BatchNorm*>(l)) return FK_BN;
  if (auto* a = dynamic_cast<const Activation*>(l)) return a->is_relu() ? FK_RELU : FK_ACT;
  if (auto* p = dynamic_cast<const Pool2D*>(l)) return p->is_max() ? FK_MAXPOOL : FK_OTHER;
  return FK_OTHER;
}

static std::vector<int> fuse_kinds(const std::vector<std::unique_ptr<Layer>>& seq) {
  std::vector<int> k;
  for (const auto& l : seq) k.push_back(fuse_kind(l.get()));
  return k;
}

// the shared planner's decisions (plan_sequence_fusions: the rules the Python layers apply too)
// wired into this sequence's layers; on = false clears every link
void fuse_bn_relu(std::vector<std::unique_ptr<Layer>>& seq, bool on) {
  const std::vector<int> f = plan_sequence_fusions(fuse_kinds(seq));
  for (size_t i = 0; i < seq.size(); ++i) {
    Layer* l = seq[i].get();
    if (auto* conv = dynamic_cast<Conv2D*>(l)) {
      // conv -> BatchNorm: the conv's epilogue emits the BatchNorm's statistics rows
      conv->set_stats_consumer(on && (f[i] & FF_EMIT_BN_STATS) ? static_cast<BatchNorm*>(seq[i + 1].get()) : nullptr);
      // BatchNorm [+ ReLU] -> conv: the conv's data gradient carries the BatchNorm backward
      BatchNorm* prod = nullptr;
      if (on && (f[i] & FF_BNB_CONSUMER))
        prod = static_cast<BatchNorm*>(seq[fuse_kind(seq[i - 1].get()) == FK_BN ? i - 1 : i - 2].get());
      conv->set_bnb_producer(prod);
    } else if (auto* bn = dynamic_cast<BatchNorm*>(l)) {
      bn->set_fused_relu(on && (f[i] & FF_FUSE_RELU));
      // BatchNorm -> ReLU -> max-pool: the pool runs inside the BatchNorm's training apply
      Pool2D* pool = on && (f[i] & FF_FUSE_POOL) ? static_cast<Pool2D*>(seq[i + 2].get()) : nullptr;
      bn->set_fused_pool(pool);
      if (pool) pool->set_fused_producer(bn);
    } else if (auto* act = dynamic_cast<Activation*>(l)) {
      act->set_passthrough(on && (f[i] & FF_PASSTHROUGH));
    } else if (auto* pool = dynamic_cast<Pool2D*>(l)) {
      if (!on || i < 2 || !(f[i - 2] & FF_FUSE_POOL)) pool->set_fused_producer(nullptr);
    }
  }
}

Tensor Activation::forward(const Tensor& x, bool training) {
  (void)training;
  if (passthrough_ && dev_.is_gpu()) return x;  // (applied by the preceding BatchNorm)
  Tensor& x_ = mbc().a;
  Tensor& y_ = mbc().b;
  check_act(x, dev_, "activation");
  Tensor y = act_empty(x.shape(), dev_);
  const long N = x.dim(0), C = x.dim(1), HW = x.dim(2) * x.dim(3);
  if (code_ == ACT_SOFTMAX) {
    if (dev_.is_gpu())
      gpu_ops::softmax_fwd(x.data(), y.data(), N * HW, (int)C);
    else
      cpu_ops::softmax_fwd(x.ptr<float>(), y.ptr<float>(), N, C, HW);
    y_ = y;
    return y;
  }
  if (dev_.is_gpu())
    gpu_ops::act_fwd(code_, x.data(), y.data(), x.numel(), act_alpha(code_));
  else
    cpu_ops::act_fwd(code_, x.ptr<float>(), y.ptr<float>(), x.numel(), act_alpha(code_));
  x_ = x;
  return y;
}

Tensor Activation::backward(const Tensor& dy) {
  if (passthrough_ && dev_.is_gpu()) return dy;
  const Tensor& x_ = mbc().a;
  const Tensor& y_ = mbc().b;
  if (code_ == ACT_SOFTMAX) {
    Tensor dx = act_empty(y_.shape(), dev_);
    const long N = y_.dim(0), C = y_.dim(1), HW = y_.dim(2) * y_.dim(3);
    if (dev_.is_gpu())
      gpu_ops::softmax_bwd(y_.data(), dy.data(), dx.data(), N * HW, (int)C);
    else
      cpu_ops::softmax_bwd(y_.ptr<float>(), dy.ptr<float>(), dx.ptr<float>(), N, C, HW);
    return dx;
  }
  Tensor dx = act_empty(x_.shape(), dev_);
  if (dev_.is_gpu())
    gpu_ops::act_bwd(code_, x_.data(), dy.data(), dx.data(), x_.numel(), act_alpha(code_));
  else
    cpu_ops::act_bwd(code_, x_.ptr<float>(), dy.ptr<float>(), dx.ptr<float>(), x_.numel(), act_alpha(code_));
  return dx;
}

// ------------------------------------------------------------------ GroupNorm
GroupNorm::GroupNorm(int num_groups, int num_channels, float eps, bool affine, std::string name)
    : Layer(std::move(name)), g_(num_groups), c_(num_channels), eps_(eps), affine_(affine) {
  if (g_ <= 0 || c_ % g_) throw std::invalid_argument("groupnorm: channels must divide into the groups");
}

json::Value GroupNorm::parameters_config() const {
  json::Value p = json::Value::object();
  p["num_groups"] = g_;
  p["num_channels"] = c_;
  p["epsilon"] = (double)eps_;
  p["affine"] = affine_;
  return p;
}

void GroupNorm::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  (void)in;
  (void)seed;
  dev_ = dev;
  params_.clear();
  // (the kernels take gamma / beta always: non-affine runs with the identity pair)
  add_param("gamma", {c_, 1, 1, 1}, Layout::NCHW, std::vector<float>((size_t)c_, 1.f));
  add_param("beta", {c_, 1, 1, 1}, Layout::NCHW, std::vector<float>((size_t)c_, 0.f));
  if (!affine_) {
    params_.clear();
    gb_identity_ = true;
  }
}

Tensor GroupNorm::forward(const Tensor& x, bool training) {
  (void)training;
  MbCache& mc = mbc();
  Tensor& x_ = mc.a;
  Tensor& mean_ = mc.b;
  Tensor& istd_ = mc.c;
  check_act(x, dev_, "groupnorm");
  if (x.dim(1) != c_) throw std::runtime_error(name_ + ": channel count mismatch");
  const long N = x.dim(0), HW = x.dim(2) * x.dim(3);
  mean_.ensure({N * g_}, DType::F32, dev_);
  istd_.ensure({N * g_}, DType::F32, dev_);
  if (!affine_ && !ident_.defined()) {
    std::vector<float> gb((size_t)2 * c_, 0.f);
    std::fill(gb.begin(), gb.begin() + c_, 1.f);
    ident_ = Tensor::from_host(gb, {2 * c_}, dev_);
  }
  const float* g = affine_ ? params_[0].value.ptr<float>() : ident_.ptr<float>();
  const float* b = affine_ ? params_[1].value.ptr<float>() : ident_.ptr<float>() + c_;
  Tensor y = act_empty(x.shape(), dev_);
  if (dev_.is_gpu())
    gpu_ops::groupnorm_fwd(x.data(), y.data(), (int)N, (int)HW, c_, g_, g, b, eps_, mean_.ptr<float>(),
                           istd_.ptr<float>());
  else
    cpu_ops::groupnorm_fwd(x.ptr<float>(), y.ptr<float>(), N, c_, HW, g_, g, b, eps_, mean_.ptr<float>(),
                           istd_.ptr<float>());
  x_ = x;
  return y;
}

Tensor GroupNorm::backward(const Tensor& dy) {
  MbCache& mc = mbc();
  const Tensor& x_ = mc.a;
  Tensor& mean_ = mc.b;
  Tensor& istd_ = mc.c;
  const long N = x_.dim(0), HW = x_.dim(2) * x_.dim(3);
  Tensor dx = act_empty(x_.shape(), dev_);
  const float* g = affine_ ? params_[0].value.ptr<float>() : ident_.ptr<float>();
  if (!affine_ && !scratch_.defined()) scratch_ = Tensor::zeros({2 * c_}, DType::F32, dev_);
  float* dg = affine_ ? params_[0].grad.ptr<float>() : scratch_.ptr<float>();
  float* db = affine_ ? params_[1].grad.ptr<float>() : scratch_.ptr<float>() + c_;
  if (dev_.is_gpu())
    gpu_ops::groupnorm_bwd(dy.data(), x_.data(), dx.data(), (int)N, (int)HW, c_, g_, g, mean_.ptr<float>(),
                           istd_.ptr<float>(), dg, db);
  else
    cpu_ops::groupnorm_bwd(x_.ptr<float>(), dy.ptr<float>(), mean_.ptr<float>(), istd_.ptr<float>(), g,
                           dx.ptr<float>(), dg, db, N, c_, HW, g_);
  return dx;
}

// ------------------------------------------------------------------ Dropout
Dropout::Dropout(float rate, std::string name) : Layer(std::move(name)), p_(rate) {
  if (!(rate >= 0.f && rate < 1.f)) throw std::invalid_argument("dropout: rate must be in [0, 1)");
}

json::Value Dropout::parameters_config() const {
  json::Value p = json::Value::object();
  p["dropout_rate"] = (double)p_;
  return p;
}

void Dropout::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  (void)in;
  dev_ = dev;
  seed_ = seed * 0x2545f4914f6cdd1dull + 0x1234567ull;
}

Tensor Dropout::forward(const Tensor& x, bool training) {
  check_act(x, dev_, "dropout");
  uint64_t& cur_ = mbc().u;
  bool& active_ = mbc().flag;
  active_ = training && p_ > 0.f;
  if (!active_) return x;
  cur_ = seed_ + 0x9e3779b97f4a7c15ull * (++draw_);  // a new mask per forward
  Tensor y = act_empty(x.shape(), dev_);
  if (dev_.is_gpu())
    gpu_ops::dropout(x.data(), y.data(), x.numel(), p_, cur_);
  else
    cpu_ops::dropout(x.ptr<float>(), y.ptr<float>(), x.numel(), p_, cur_);
  return y;
}

Tensor Dropout::backward(const Tensor& dy) {
  const uint64_t cur_ = mbc().u;
  const bool active_ = mbc().flag;
  if (!active_) return dy;
  Tensor dx = act_empty(dy.shape(), dev_);
  if (dev_.is_gpu())
    gpu_ops::dropout(dy.data(), dx.data(), dy.numel(), p_, cur_);  // the forward's mask and scale
  else
    cpu_ops::dropout(dy.ptr<float>(), dx.ptr<float>(), dy.numel(), p_, cur_);
  return dx;
}

// ------------------------------------------------------------------ ResidualBlock
ResidualBlock::ResidualBlock(std::vector<std::unique_ptr<Layer>> main, std::vector<std::unique_ptr<Layer>> shortcut,
                             std::string activation, std::string name)
    : Layer(std::move(name)), main_(std::move(main)), short_(std::move(shortcut)), act_(std::move(activation)) {
  if (act_ != "relu" && act_ != "none" && act_ != "linear")
    throw std::invalid_argument("residual_block: activation must be relu, none or linear");
}

static json::Value path_config(const std::vector<std::unique_ptr<Layer>>& path) {
  json::Value arr = json::Value::array();
  for (auto& l : path) {
    json::Value r = json::Value::object();
    r["type"] = l->type();
    r["name"] = l->name();
    r["parameters"] = l->parameters_config();
    arr.push(std::move(r));
  }
  return arr;
}

json::Value ResidualBlock::parameters_config() const {
  json::Value p = json::Value::object();
  p["activation"] = act_;
  p["has_projection"] = !short_.empty();
  p["main_path"] = path_config(main_).dump();
  p["shortcut_path"] = path_config(short_).dump();
  return p;
}

std::vector<int64_t> ResidualBlock::output_shape(const std::vector<int64_t>& in) const {
  std::vector<int64_t> s = in;
  for (auto& l : main_) s = l->output_shape(s);
  return s;
}

void ResidualBlock::build(const std::vector<int64_t>& in, Device dev, uint64_t seed) {
  dev_ = dev;
  fuse_bn_relu(main_, dev.is_gpu());
  fuse_bn_relu(short_, dev.is_gpu());
  std::vector<int64_t> s = in;
  uint64_t k = 0;
  for (auto& l : main_) {
    l->build(s, dev, seed * 31ull + (k++) * 104729ull);
    if (s[1] > 0) s = l->output_shape(s);
  }
  s = in;
  for (auto& l : short_) {
    l->build(s, dev, seed * 31ull + (k++) * 104729ull);
    if (s[1] > 0) s = l->output_shape(s);
  }
}

double ResidualBlock::flops(const std::vector<int64_t>& in) const {
  double f = 0;
  std::vector<int64_t> s = in;
  for (auto& l : main_) {
    f += l->flops(s);
    s = l->output_shape(s);
  }
  std::vector<int64_t> t = in;
  for (auto& l : short_) {
    f += l->flops(t);
    t = l->output_shape(t);
  }
  return f + 2.0 * (double)s[0] * (double)s[1] * (double)s[2] * (double)s[3];  // the join
}

Conv2D* ResidualBlock::head_conv() const { return main_.empty() ? nullptr : dynamic_cast<Conv2D*>(main_[0].get()); }

void fuse_blocks(std::vector<std::unique_ptr<Layer>>& seq, bool on) {
  for (size_t i = 0; i + 1 < seq.size(); ++i) {
    auto* prev = dynamic_cast<ResidualBlock*>(seq[i].get());
    auto* next = dynamic_cast<ResidualBlock*>(seq[i + 1].get());
    if (prev == nullptr || next == nullptr) continue;
    BatchNorm* tail = prev->fused_tail();
    Conv2D* head = next->head_conv();
    if (head == nullptr) continue;
    head->set_block_bnb_producer(on && tail != nullptr && next->fused_tail() != nullptr ? tail : nullptr);
  }
}

// the shared planner's residual rules (plan_residual_fusions; the Python ResidualBlock too)
BatchNorm* ResidualBlock::dual_shortcut() const {
  if (!dev_.is_gpu() ||
      !(plan_residual_fusions(fuse_kinds(main_), fuse_kinds(short_), act_ == "relu" || act_ == "linear") &
        RF_DUAL_SHORTCUT))
    return nullptr;
  return static_cast<BatchNorm*>(short_.back().get());
}

BatchNorm* ResidualBlock::fused_tail() const {
  if (!dev_.is_gpu() ||
      !(plan_residual_fusions(fuse_kinds(main_), fuse_kinds(short_), act_ == "relu" || act_ == "linear") &
        RF_FUSED_TAIL))
    return nullptr;
  return static_cast<BatchNorm*>(main_.back().get());
}

Tensor ResidualBlock::forward(const Tensor& x, bool training) {
  check_act(x, dev_, "residual_block");
  Tensor& y_ = mbc().a;
  if (BatchNorm* tail = fused_tail()) {  // y = act(bn(main(x)) + shortcut(x)) in the BN's apply pass
    // a projection shortcut's closing BatchNorm is applied inside the same pass (forward_dual):
    // its statistics rows are taken now (the shortcut conv's slab in the secondary workspace, so
    // the main path's convs leave it intact), its normalised output is never written
    BatchNorm* sbn = dual_shortcut();
    Tensor sc = x;
    {
      std::unique_ptr<gpu_ops::SecondaryStats> alt(sbn ? new gpu_ops::SecondaryStats() : nullptr);
      for (size_t i = 0; i + (sbn ? 1 : 0) < short_.size(); ++i) sc = short_[i]->forward(sc, training);
    }
    if (sbn) sbn->forward_deferred(sc, training);
    Tensor m = x;
    for (size_t i = 0; i + 1 < main_.size(); ++i) m = main_[i]->forward(m, training);
    if (m.shape() != sc.shape())
      throw std::runtime_error(name_ + ": main path " + shape_str(m.shape()) + " vs shortcut " + shape_str(sc.shape()));
    y_ = sbn ? tail->forward_dual(m, *sbn, act_ == "relu", training)
             : tail->forward_residual(m, sc, act_ == "relu", training);
    return y_;
  }
  Tensor m = x;
  for (auto& l : main_) m = l->forward(m, training);
  Tensor sc = x;
  for (auto& l : short_) sc = l->forward(sc, training);
  if (m.shape() != sc.shape())
    throw std::runtime_error(name_ + ": main path " + shape_str(m.shape()) + " vs shortcut " + shape_str(sc.shape()));
  Tensor y = act_empty(m.shape(), dev_);
  const bool relu = act_ == "relu";
  if (dev_.is_gpu())
    gpu_ops::add(m.data(), sc.data(), y.data(), y.numel(), relu);
  else
    cpu_ops::add(m.ptr<float>(), sc.ptr<float>(), y.ptr<float>(), y.numel(), relu);
  y_ = y;
  return y;
}

Tensor ResidualBlock::backward(const Tensor& dy) {
  const Tensor& y_ = mbc().a;
  if (BatchNorm* tail = fused_tail()) {
    Tensor gs, gm;  // gs: the activation-masked dy, for the shortcut
    BatchNorm* sbn = dual_shortcut();
    if (sbn != nullptr && tail->backward_dual(dy, *sbn, gm, gs)) {
      // both BatchNorms' data gradients from one pass; gs is already below the shortcut BatchNorm
      for (size_t i = short_.size() - 1; i-- > 0;) gs = short_[i]->backward(gs);
    } else {
      gm = tail->backward_residual(dy, &gs);
      for (size_t i = short_.size(); i-- > 0;) gs = short_[i]->backward(gs);
    }
    for (size_t i = main_.size() - 1; i-- > 1;) gm = main_[i]->backward(gm);
    // the main path's first conv adds the shortcut gradient in its data-gradient epilogue
    auto* head = dynamic_cast<Conv2D*>(main_[0].get());
    if (head != nullptr && input_grad_ && gs.defined() && gs.dtype() == DType::BF16) return head->backward_residual(gm, gs);
    gm = main_[0]->backward(gm);
    if (!gm.defined() || !gs.defined()) return Tensor();
    Tensor dx = act_empty(gm.shape(), dev_);
    gpu_ops::add(gm.data(), gs.data(), dx.data(), dx.numel(), false);
    return dx;
  }
  Tensor g = dy;
  if (act_ == "relu") {
    g = act_empty(dy.shape(), dev_);
    if (dev_.is_gpu())
      gpu_ops::relu_mask(dy.data(), y_.data(), g.data(), dy.numel());
    else
      cpu_ops::relu_mask(dy.ptr<float>(), y_.ptr<float>(), g.ptr<float>(), dy.numel());
  }
  Tensor gm = g;
  for (size_t i = main_.size(); i-- > 0;) gm = main_[i]->backward(gm);
  Tensor gs = g;
  for (size_t i = short_.size(); i-- > 0;) gs = short_[i]->backward(gs);
  Tensor dx = act_empty(gm.shape(), dev_);
  if (dev_.is_gpu())
    gpu_ops::add(gm.data(), gs.data(), dx.data(), dx.numel(), false);
  else
    cpu_ops::add(gm.ptr<float>(), gs.ptr<float>(), dx.ptr<float>(), dx.numel(), false);
  return dx;
}

void ResidualBlock::set_micro_batch(int mb) {
  mb_ = mb;
  for (auto& l : main_) l->set_micro_batch(mb);
  for (auto& l : short_) l->set_micro_batch(mb);
}

void ResidualBlock::sync_shadow() {
  for (auto& l : main_) l->sync_shadow();
  for (auto& l : short_) l->sync_shadow();
}

void ResidualBlock::collect_params(std::vector<Param*>& out) {
  for (auto& l : main_) l->collect_params(out);
  for (auto& l : short_) l->collect_params(out);
}

void ResidualBlock::collect_layers(std::vector<Layer*>& out) {
  out.push_back(this);
  for (auto& l : main_) l->collect_layers(out);
  for (auto& l : short_) l->collect_layers(out);
}

// ------------------------------------------------------------------ pooling
Pool2D::Pool2D(bool max, int kh, int kw, int sh, int sw, int ph, int pw, std::string name)
    : Layer(std::move(name)), max_(max), kh_(kh), kw_(kw), sh_(sh > 0 ? sh : kh), sw_(sw > 0 ? sw : kw), ph_(ph),
      pw_(pw) {}

json::Value Pool2D::parameters_config() const {
  json::Value p = json::Value::object();
  p["pool_h"] = kh_;
  p["pool_w"] = kw_;
  p["stride_h"] = sh_;
  p["stride_w"] = sw_;
  p["pad_h"] = ph_;
  p["pad_w"] = pw_;
  return p;
}

PoolShape Pool2D::shape_for(const std::vector<int64_t>& in) const {
  PoolShape p{};
  p.N = (int)in[0];
  p.C = (int)in[1];
  p.H = (int)in[2];
  p.W = (int)in[3];
  p.KH = kh_;
  p.KW = kw_;
  p.SH = sh_;
  p.SW = sw_;
  p.PH = ph_;
  p.PW = pw_;
  p.OH = (p.H + 2 * ph_ - kh_) / sh_ + 1;
  p.OW = (p.W + 2 * pw_ - kw_) / sw_ + 1;
  return p;
}

std::vector<int64_t> Pool2D::output_shape(const std::vector<int64_t>& in) const {
  const PoolShape p = shape_for(in);
  return {in[0], in[1], p.OH, p.OW};
}

uint8_t* Pool2D::accept_prepooled(const Tensor& ypool, const std::vector<int64_t>& in) {
  MbCache& mc = mbc();
  const PoolShape p = shape_for(in);
  mc.a.ensure({(int64_t)p.N * p.C * p.OH * p.OW}, DType::U8, dev_);
  mc.b = ypool;
  mc.shape = in;
  mc.flag = true;
  return mc.a.ptr<uint8_t>();
}

Tensor Pool2D::forward(const Tensor& x, bool training) {
  (void)training;
  if (bn_ != nullptr && mbc().flag && mbc().b.defined() && mbc().b.data() == x.data())
    return x;  // computed by the fused BatchNorm + ReLU (accept_prepooled)
  mbc().flag = false;
  Tensor& idx_ = mbc().a;
  std::vector<int64_t>& in_shape_ = mbc().shape;
  check_act(x, dev_, "pool2d");
  const PoolShape p = shape_for(x.shape());
  Tensor y = act_empty({p.N, p.C, p.OH, p.OW}, dev_);
  in_shape_ = x.shape();
  if (max_) {
    const int64_t n = (int64_t)p.N * p.C * p.OH * p.OW;
    if (dev_.is_gpu()) {
      idx_.ensure({n}, DType::U8, dev_);
      gpu_ops::maxpool_fwd(x.data(), y.data(), idx_.ptr<uint8_t>(), p);
    } else {
      idx_.ensure({n}, DType::I32, dev_);
      cpu_ops::maxpool_fwd(x.ptr<float>(), y.ptr<float>(), idx_.ptr<int32_t>(), p);
    }
  } else if (dev_.is_gpu()) {
    gpu_ops::avgpool_fwd(x.data(), y.data(), p);
  } else {
    cpu_ops::avgpool_fwd(x.ptr<float>(), y.ptr<float>(), p);
  }
  return y;
}

Tensor Pool2D::backward(const Tensor& dy) {
  const Tensor& idx_ = mbc().a;
  const std::vector<int64_t>& in_shape_ = mbc().shape;
  const PoolShape p = shape_for(in_shape_);
  Tensor dx = act_empty(in_shape_, dev_);
  if (mbc().flag && bn_ != nullptr) {
    // masked with the pooled value (y > 0) and the BatchNorm's backward statistics in the same
    // pass; the BatchNorm's backward picks them up (offer_bwd_stats)
    const gpu_ops::BnbOperands ops = bn_->bnb_operands(mb_);
    int rows = 0;
    const float* slab = gpu_ops::maxpool_bwd_bnb(dy.data(), idx_.ptr<uint8_t>(), mbc().b.data(), ops.x, ops.mean,
                                                 ops.istd, dx.data(), p, &rows);
    bn_->offer_bwd_stats(dx.data(), slab, rows);
    return dx;
  }
  if (max_) {
    if (dev_.is_gpu())
      gpu_ops::maxpool_bwd(dy.data(), idx_.ptr<uint8_t>(), dx.data(), p);
    else
      cpu_ops::maxpool_bwd(dy.ptr<float>(), idx_.ptr<int32_t>(), dx.ptr<float>(), p);
  } else if (dev_.is_gpu()) {
    gpu_ops::avgpool_bwd(dy.data(), dx.data(), p);
  } else {
    cpu_ops::avgpool_bwd(dy.ptr<float>(), dx.ptr<float>(), p);
  }
  return dx;
}

// ------------------------------------------------------------------ Flatten
std::vector<int64_t> Flatten::output_shape(const std::vector<int64_t>& in) const {
  return {in[0], in[1] * in[2] * in[3], 1, 1};
}

Tensor Flatten::forward(const Tensor& x, bool training) {
  (void)training;
  std::vector<int64_t>& in_shape_ = mbc().shape;
  check_act(x, dev_, "flatten");
  in_shape_ = x.shape();
  const auto os = output_shape(x.shape());
  const int64_t HW = x.dim(2) * x.dim(3);
  if (!dev_.is_gpu()) return x.view(os);            // NCHW: already in feature order
  if (HW == 1) return x.view(os, Layout::NHWC);     // nothing to reorder
  Tensor y = act_empty(os, dev_);
  gpu_ops::nhwc_to_nchw(x.data(), y.data(), (int)x.dim(0), (int)HW, (int)x.dim(1));  // NCHW feature order
  return y;
}

Tensor Flatten::backward(const Tensor& dy) {
  const std::vector<int64_t>& in_shape_ = mbc().shape;
  const int64_t HW = in_shape_[2] * in_shape_[3];
  if (!dev_.is_gpu()) return dy.view(in_shape_);
  if (HW == 1) return dy.view(in_shape_, Layout::NHWC);
  Tensor dx = act_empty(in_shape_, dev_);
  gpu_ops::nchw_to_nhwc_bf16(dy.data(), dx.data(), (int)in_shape_[0], (int)HW, (int)in_shape_[1]);
  return dx;
}

// ------------------------------------------------------------------ factory
std::unique_ptr<Layer> create_layer(const json::Value& rec) {
  const std::string type = rec.get_string("type", "");
  const std::string name = rec.get_string("name", type);
  static const json::Value empty = json::Value::object();
  const json::Value& p = rec.has("parameters") ? rec.at("parameters") : empty;
  auto I = [&](const char* k, int64_t d) { return (int)p.get_int(k, d); };
  if (type == "conv2d")
    return std::make_unique<Conv2D>(I("in_channels", 0), I("out_channels", 0), I("kernel_h", 1), I("kernel_w", 1),
                                    I("stride_h", 1), I("stride_w", 1), I("pad_h", 0), I("pad_w", 0),
                                    p.get_bool("use_bias", true), name);
  if (type == "dense")
    return std::make_unique<Dense>(I("input_features", 0), I("output_features", 0), p.get_bool("use_bias", true),
                                   name);
  if (type == "batchnorm")
    return std::make_unique<BatchNorm>(I("num_features", 0), (float)p.get_number("epsilon", 1e-5),
                                       (float)p.get_number("momentum", 0.1), p.get_bool("affine", true), name);
  if (type == "activation") return std::make_unique<Activation>(p.get_string("activation", "relu"), name);
  if (type == "maxpool2d" || type == "avgpool2d")
    return std::make_unique<Pool2D>(type == "maxpool2d", I("pool_h", 2), I("pool_w", 2), I("stride_h", 0),
                                    I("stride_w", 0), I("pad_h", 0), I("pad_w", 0), name);
  if (type == "flatten") return std::make_unique<Flatten>(name);
  if (type == "groupnorm")
    return std::make_unique<GroupNorm>(I("num_groups", 1), I("num_channels", 0), (float)p.get_number("epsilon", 1e-5),
                                       p.get_bool("affine", true), name);
  if (type == "dropout") return std::make_unique<Dropout>((float)p.get_number("dropout_rate", 0.5), name);
  if (type == "residual_block") {
    auto path = [&](const char* key) {
      std::vector<std::unique_ptr<Layer>> out;
      const std::string txt = p.get_string(key, "[]");
      const json::Value arr = json::Value::parse(txt.empty() ? "[]" : txt);  // (kept alive for the loop)
      for (auto& r : arr.items()) out.push_back(create_layer(r));
      return out;
    };
    auto main = path("main_path");
    std::vector<std::unique_ptr<Layer>> sc;
    if (p.get_bool("has_projection", false)) sc = path("shortcut_path");
    return std::make_unique<ResidualBlock>(std::move(main), std::move(sc), p.get_string("activation", "relu"), name);
  }
  throw std::invalid_argument("C++ host API: unsupported layer type '" + type + "'");
}

// ------------------------------------------------------------------ Sequential
namespace {
// host fp32 values (logical order) into an existing parameter tensor's storage
void assign_values(Tensor& dst, const std::vector<float>& v, const std::vector<int64_t>& shape, Layout layout) {
  const Tensor h = Tensor::from_host(v, shape, Device::cpu(), DType::F32, layout);
  if (h.nbytes() != dst.nbytes()) throw std::runtime_error("parameter size mismatch");
  if (dst.device().is_gpu())
    gpu::copy(dst.data(), h.data(), h.nbytes(), 0);
  else
    std::memcpy(dst.data(), h.data(), h.nbytes());
}
}  // namespace

void Sequential::pack_params() {
  arena_.reset();
  std::vector<Param*> ps = parameters();
  if (ps.empty() || !dev_.is_gpu()) return;
  auto A = std::make_shared<ParamArena>();
  std::vector<size_t> off;
  for (Param* p : ps) {
    off.push_back(A->n);
    A->n += ((size_t)p->value.numel() + 63) / 64 * 64;
  }
  A->count = ps.size();
  const int64_t n = (int64_t)A->n;
  A->value = Tensor::zeros({n}, DType::F32, dev_);
  A->grad = Tensor::zeros({n}, DType::F32, dev_);
  A->m = Tensor::zeros({n}, DType::F32, dev_);
  A->v = Tensor::zeros({n}, DType::F32, dev_);
  A->shadow = Tensor::zeros({n}, DType::BF16, dev_);
  for (size_t k = 0; k < ps.size(); ++k) {
    Param* p = ps[k];
    const auto& sh = p->value.shape();
    const Layout lay = p->value.layout();
    Tensor nv = A->value.slice(off[k] * 4, sh, DType::F32, lay);
    gpu::copy(nv.data(), p->value.data(), p->value.nbytes(), 2);
    p->value = nv;
    p->grad = A->grad.slice(off[k] * 4, sh, DType::F32, lay);
    p->m = A->m.slice(off[k] * 4, sh, DType::F32, lay);
    p->v = A->v.slice(off[k] * 4, sh, DType::F32, lay);
    Tensor ns = A->shadow.slice(off[k] * 2, sh, DType::BF16, lay);
    if (p->shadow.defined()) gpu::copy(ns.data(), p->shadow.data(), p->shadow.nbytes(), 2);
    p->shadow = ns;
    p->arena = A;
  }
  // the convs' pre-transposed dgrad operands (from the arena shadows)
  std::vector<Layer*> all;
  for (auto& l : layers_) l->collect_layers(all);
  std::vector<int64_t> table;
  for (Layer* l : all) {
    auto* c = dynamic_cast<Conv2D*>(l);
    std::vector<int64_t> row;
    long tiles = 0;
    if (c == nullptr || !c->make_transposed_operand(row, tiles)) continue;
    table.insert(table.end(), row.begin(), row.end());
    ++A->n_wt;
    A->wt_tiles = std::max(A->wt_tiles, tiles);
  }
  if (A->n_wt) {
    A->wt_table = Tensor::empty({(int64_t)table.size()}, DType::I64, dev_);
    gpu::copy(A->wt_table.data(), table.data(), table.size() * 8, 0);
    A->refresh_transposes();
  }
  arena_ = A;
}

void Sequential::set_device(Device d) {
  if (d.is_gpu() && gpu::device_count() <= d.index) throw std::runtime_error(d.str() + " not available");
  if (initialized_ && d != dev_) {
    // move: rebuild on the new device with the current values
    std::vector<std::vector<float>> vals;
    for (auto* p : parameters()) vals.push_back(p->value.to_host_f32());
    dev_ = d;
    initialized_ = false;
    initialize(0);
    size_t i = 0;
    for (auto* p : parameters()) assign_values(p->value, vals[i++], p->shape, p->layout);
    for (auto& l : layers_) l->sync_shadow();
    return;
  }
  dev_ = d;
}

void Sequential::initialize(uint64_t seed) {
  if (input_chw_.empty()) {
    // infer the input channels from the first parameterised layer (spatial size is not needed to
    // create parameters)
    input_chw_ = {0, 0, 0};
  }
  std::vector<int64_t> shape{1, input_chw_[0], input_chw_[1], input_chw_[2]};
  fuse_bn_relu(layers_, dev_.is_gpu());
  uint64_t k = 0;
  for (auto& l : layers_) {
    l->build(shape, dev_, seed * 1000003ull + (k++) * 7919ull);
    if (shape[1] > 0 && shape[2] > 0) shape = l->output_shape(shape);
  }
  fuse_blocks(layers_, dev_.is_gpu());
  pack_params();
  initialized_ = true;
}

std::vector<Param*> Sequential::parameters() {
  std::vector<Param*> out;
  for (auto& l : layers_) l->collect_params(out);
  return out;
}

std::vector<BatchNorm*> Sequential::batchnorms() {
  std::vector<Layer*> all;
  for (auto& l : layers_) l->collect_layers(all);
  std::vector<BatchNorm*> out;
  for (auto* l : all)
    if (auto* bn = dynamic_cast<BatchNorm*>(l)) out.push_back(bn);
  return out;
}

size_t Sequential::num_parameters() {
  size_t n = 0;
  for (auto* p : parameters()) n += (size_t)p->value.numel();
  return n;
}

void Sequential::zero_grad() {
  if (arena_) {
    gpu_ops::zero(arena_->grad.data(), (long)arena_->grad.nbytes());
    return;
  }
  for (auto* p : parameters()) {
    if (dev_.is_gpu())
      gpu_ops::zero(p->grad.data(), (long)p->grad.nbytes());
    else
      p->grad.zero_();
  }
}

std::vector<double> Sequential::layer_flops(const std::vector<int64_t>& in) const {
  std::vector<double> out;
  std::vector<int64_t> s = in;
  for (auto& l : layers_) {
    out.push_back(l->flops(s));
    s = l->output_shape(s);
  }
  return out;
}

Tensor Sequential::input_activation(const Tensor& x_in) const {
  if (x_in.rank() != 4 || x_in.dtype() != DType::F32) throw std::runtime_error("forward: expected fp32 (N, C, H, W)");
  Tensor x = x_in.device() == dev_ ? x_in : x_in.to(dev_);
  if (dev_.is_gpu() && !layers_.empty() && layers_[0]->takes_raw_input(x.shape())) return x;  // (RGB stem)
  if (dev_.is_gpu()) {
    Tensor a = Tensor::empty(x.shape(), DType::BF16, dev_, Layout::NHWC);
    gpu_ops::input_to_nhwc(x.ptr<float>(), a.data(), (int)x.dim(0), (int)x.dim(1), (int)(x.dim(2) * x.dim(3)));
    x = a;
  }
  return x;
}

Tensor Sequential::forward_activation(const Tensor& x_in, int mb) {
  if (!initialized_) throw std::runtime_error("Sequential::forward before initialize()");
  Tensor x = x_in;
  for (auto& l : layers_) {
    l->set_micro_batch(mb);
    x = l->forward(x, training_);
  }
  return x;
}

Tensor Sequential::backward_activation(const Tensor& g_in, int mb) {
  Tensor g = g_in;
  // (DCNN_DEFER_REDUCE=0: each weight gradient's split-K reduce right after its kernel — experiment)
  static const bool defer_env = [] {
    const char* v = std::getenv("DCNN_DEFER_REDUCE");
    return !(v && std::string(v) == "0");
  }();
  const bool defer = dev_.is_gpu() && defer_env;
  // (DCNN_STEM_BN_FOLD=0: the stem BatchNorm's backward as its own pass — test / A-B hook)
  static const bool stem_bn_env = [] {
    const char* v = std::getenv("DCNN_STEM_BN_FOLD");
    return !(v && std::string(v) == "0");
  }();
  const bool stem_bn_fold = dev_.is_gpu() && stem_bn_env && layers_.size() > 1;
  if (defer) gpu_ops::begin_deferred_reduce();
  try {
    for (size_t i = layers_.size(); i-- > 0;) {
      layers_[i]->set_micro_batch(mb);
      if (i == 1 && stem_bn_fold) {
        // the RGB stem's BatchNorm backward inside the stem's weight-gradient kernel (its input
        // gradient, a full-resolution pass written and read once, is never materialised)
        auto* bn = dynamic_cast<BatchNorm*>(layers_[1].get());
        auto* conv = dynamic_cast<Conv2D*>(layers_[0].get());
        if (bn && conv) {
          conv->set_micro_batch(mb);
          if (bn->backward_into_stem(g, *conv)) {
            if (bwd_hook_) bwd_hook_(1);
            if (bwd_hook_) bwd_hook_(0);
            g = Tensor();
            break;
          }
        }
      }
      g = layers_[i]->backward(g);
      if (bwd_hook_) bwd_hook_(i);
    }
  } catch (...) {
    if (defer) gpu_ops::end_deferred_reduce();
    throw;
  }
  if (defer) gpu_ops::end_deferred_reduce();  // every weight gradient final before the optimizer
  return g;
}

Tensor Sequential::forward(const Tensor& x_in, int mb) {
  Tensor x = forward_activation(input_activation(x_in), mb);
  return x.view({x.dim(0), x.dim(1) * x.dim(2) * x.dim(3)}, x.layout());
}

void Sequential::backward(const Tensor& dlogits, int mb) {
  if (!layers_.empty()) layers_[0]->set_input_grad(false);  // (nothing consumes d loss / d input)
  Tensor g = dlogits.view({dlogits.dim(0), dlogits.dim(1), 1, 1}, dev_.is_gpu() ? Layout::NHWC : Layout::NCHW);
  backward_activation(g, mb);
}

json::Value Sequential::get_config() const {
  json::Value c = json::Value::object();
  c["name"] = name_;
  c["is_training"] = training_;
  json::Value ls = json::Value::array();
  for (auto& l : layers_) {
    json::Value r = json::Value::object();
    r["type"] = l->type();
    r["name"] = l->name();
    r["parameters"] = l->parameters_config();
    ls.push(std::move(r));
  }
  c["layers"] = std::move(ls);
  if (!input_chw_.empty() && input_chw_[0] > 0) {
    json::Value in = json::Value::array();
    for (auto v : input_chw_) in.push(v);
    c["input_shape"] = std::move(in);
  }
  return c;
}

void Sequential::print_config() const { std::cout << get_config().dump(2) << std::endl; }

Sequential Sequential::load_from_config(const json::Value& cfg) {
  Sequential m(cfg.get_string("name", "sequential"));
  for (auto& r : cfg.at("layers").items()) m.add(create_layer(r));
  m.set_training(cfg.get_bool("is_training", true));
  if (const json::Value* in = cfg.find("input_shape")) {
    std::vector<int64_t> chw;
    for (auto& v : in->items()) chw.push_back(v.as_int());
    m.set_input_shape(chw);
  }
  return m;
}

void Sequential::save_to_file(const std::string& path) const {
  const std::filesystem::path dir = std::filesystem::path(path).parent_path();
  if (!dir.empty()) std::filesystem::create_directories(dir);
  {
    std::ofstream f(path + ".json");
    if (!f) throw std::runtime_error("cannot write " + path + ".json");
    f << get_config().dump(4);
  }
  std::ofstream f(path + ".bin", std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path + ".bin");
  auto& self = const_cast<Sequential&>(*this);
  for (auto* p : self.parameters()) p->value.view(p->shape, p->layout).save(f);
  // BatchNorm running statistics: language-neutral sidecar of .bin records (running_mean,
  // running_var per BatchNorm in depth-first layer order), read by both front ends
  std::ofstream s(path + ".bnstats", std::ios::binary);
  for (auto* bn : self.batchnorms()) {
    const int64_t c = bn->running_mean.numel();
    bn->running_mean.view({c, 1, 1, 1}).save(s);
    bn->running_var.view({c, 1, 1, 1}).save(s);
  }
}

void Sequential::load_bn_stats(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  for (auto* bn : batchnorms()) {
    const int64_t c = bn->running_mean.numel();
    Tensor m = Tensor::load(f), v = Tensor::load(f);
    if (m.numel() != c || v.numel() != c) throw std::runtime_error("bnstats: channel count mismatch");
    bn->running_mean = Tensor::from_host(m.to_host_f32(), {c}, dev_);
    bn->running_var = Tensor::from_host(v.to_host_f32(), {c}, dev_);
  }
}

void Sequential::load_weights_file(const std::string& path) {
  if (!initialized_) initialize(0);
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  for (auto* p : parameters()) {
    Tensor t = Tensor::load(f);
    if (t.numel() != p->value.numel())
      throw std::runtime_error("checkpoint tensor " + shape_str(t.shape()) + " does not match parameter " +
                               shape_str(p->shape));
    assign_values(p->value, t.to_host_f32(), p->shape, p->layout);
  }
  for (auto& l : layers_) l->sync_shadow();
}

Sequential Sequential::from_file(const std::string& path, Device dev) {
  std::ifstream f(path + ".json");
  if (!f) throw std::runtime_error("cannot read " + path + ".json");
  std::stringstream ss;
  ss << f.rdbuf();
  Sequential m = load_from_config(json::Value::parse(ss.str()));
  m.set_device(dev);
  m.initialize(0);
  m.load_weights_file(path + ".bin");
  if (std::ifstream(path + ".bnstats").good()) m.load_bn_stats(path + ".bnstats");
  return m;
}

// ------------------------------------------------------------------ builder
std::string SequentialBuilder::auto_name(const std::string& given, const std::string& kind) {
  ++count_;
  return given.empty() ? kind + "_" + std::to_string(count_) : given;
}

SequentialBuilder& SequentialBuilder::input(const std::vector<int64_t>& chw) {
  if (chw.size() != 3) throw std::invalid_argument("input: expected {C, H, W}");
  cur_ = chw;
  model_.set_input_shape(chw);
  return *this;
}

SequentialBuilder& SequentialBuilder::conv2d(int out_ch, int kh, int kw, int sh, int sw, int ph, int pw, bool bias,
                                             const std::string& name) {
  if (cur_.empty()) throw std::logic_error("SequentialBuilder: call input() first");
  auto l = std::make_unique<Conv2D>((int)cur_[0], out_ch, kh, kw, sh, sw, ph, pw, bias, auto_name(name, "conv2d"));
  const auto o = l->output_shape({1, cur_[0], cur_[1], cur_[2]});
  cur_ = {o[1], o[2], o[3]};
  model_.add(std::move(l));
  return *this;
}

SequentialBuilder& SequentialBuilder::batchnorm(float eps, float momentum, bool affine, const std::string& name) {
  model_.add(std::make_unique<BatchNorm>((int)cur_.at(0), eps, momentum, affine, auto_name(name, "batchnorm")));
  return *this;
}

SequentialBuilder& SequentialBuilder::activation(const std::string& kind, const std::string& name) {
  model_.add(std::make_unique<Activation>(kind, auto_name(name, kind)));
  return *this;
}

SequentialBuilder& SequentialBuilder::maxpool2d(int kh, int kw, int sh, int sw, int ph, int pw,
                                                const std::string& name) {
  auto l = std::make_unique<Pool2D>(true, kh, kw, sh, sw, ph, pw, auto_name(name, "maxpool2d"));
  const auto o = l->output_shape({1, cur_.at(0), cur_[1], cur_[2]});
  cur_ = {o[1], o[2], o[3]};
  model_.add(std::move(l));
  return *this;
}

SequentialBuilder& SequentialBuilder::avgpool2d(int kh, int kw, int sh, int sw, int ph, int pw,
                                                const std::string& name) {
  auto l = std::make_unique<Pool2D>(false, kh, kw, sh, sw, ph, pw, auto_name(name, "avgpool2d"));
  const auto o = l->output_shape({1, cur_.at(0), cur_[1], cur_[2]});
  cur_ = {o[1], o[2], o[3]};
  model_.add(std::move(l));
  return *this;
}

SequentialBuilder& SequentialBuilder::flatten(const std::string& name) {
  model_.add(std::make_unique<Flatten>(auto_name(name, "flatten")));
  cur_ = {cur_.at(0) * cur_[1] * cur_[2], 1, 1};
  return *this;
}

SequentialBuilder& SequentialBuilder::dense(int out_features, bool bias, const std::string& name) {
  const int in = (int)(cur_.at(0) * cur_[1] * cur_[2]);
  model_.add(std::make_unique<Dense>(in, out_features, bias, auto_name(name, "dense")));
  cur_ = {out_features, 1, 1};
  return *this;
}

SequentialBuilder& SequentialBuilder::groupnorm(int num_groups, float eps, bool affine, const std::string& name) {
  model_.add(std::make_unique<GroupNorm>(num_groups, (int)cur_.at(0), eps, affine, auto_name(name, "groupnorm")));
  return *this;
}

SequentialBuilder& SequentialBuilder::dropout(float rate, const std::string& name) {
  model_.add(std::make_unique<Dropout>(rate, auto_name(name, "dropout")));
  return *this;
}

SequentialBuilder& SequentialBuilder::residual(std::vector<std::unique_ptr<Layer>> main,
                                               std::vector<std::unique_ptr<Layer>> shortcut,
                                               const std::string& activation, const std::string& name) {
  auto l = std::make_unique<ResidualBlock>(std::move(main), std::move(shortcut), activation,
                                           auto_name(name, "residual_block"));
  const auto o = l->output_shape({1, cur_.at(0), cur_[1], cur_[2]});
  cur_ = {o[1], o[2], o[3]};
  model_.add(std::move(l));
  return *this;
}

SequentialBuilder& SequentialBuilder::basic_residual_block(int in_ch, int out_ch, int stride, const std::string& name) {
  std::vector<std::unique_ptr<Layer>> m, sc;
  m.push_back(std::make_unique<Conv2D>(in_ch, out_ch, 3, 3, stride, stride, 1, 1, true, "conv2d_0"));
  m.push_back(std::make_unique<BatchNorm>(out_ch, 1e-5f, 0.1f, true, "bn0"));
  m.push_back(std::make_unique<Activation>("relu", "relu_0"));
  m.push_back(std::make_unique<Conv2D>(out_ch, out_ch, 3, 3, 1, 1, 1, 1, true, "conv2d_1"));
  m.push_back(std::make_unique<BatchNorm>(out_ch, 1e-5f, 0.1f, true, "bn0"));
  if (stride != 1 || in_ch != out_ch) {
    sc.push_back(std::make_unique<Conv2D>(in_ch, out_ch, 1, 1, stride, stride, 0, 0, false, "conv2d_0"));
    sc.push_back(std::make_unique<BatchNorm>(out_ch, 1e-5f, 0.1f, true, "bn0"));
  }
  return residual(std::move(m), std::move(sc), "relu",
                  name.empty() ? "basic_residual_block_" + std::to_string(model_.layers().size()) : name);
}

SequentialBuilder& SequentialBuilder::bottleneck_residual_block(int in_ch, int mid_ch, int out_ch, int stride,
                                                                const std::string& name) {
  std::vector<std::unique_ptr<Layer>> m, sc;
  m.push_back(std::make_unique<Conv2D>(in_ch, mid_ch, 1, 1, 1, 1, 0, 0, false, "conv2d_0"));
  m.push_back(std::make_unique<BatchNorm>(mid_ch, 1e-3f, 0.1f, true, "bn0"));
  m.push_back(std::make_unique<Activation>("relu", "relu_0"));
  m.push_back(std::make_unique<Conv2D>(mid_ch, mid_ch, 3, 3, stride, stride, 1, 1, false, "conv2d_1"));
  m.push_back(std::make_unique<BatchNorm>(mid_ch, 1e-3f, 0.1f, true, "bn0"));
  m.push_back(std::make_unique<Activation>("relu", "relu_1"));
  m.push_back(std::make_unique<Conv2D>(mid_ch, out_ch, 1, 1, 1, 1, 0, 0, false, "conv2d_2"));
  m.push_back(std::make_unique<BatchNorm>(out_ch, 1e-3f, 0.1f, true, "bn0"));
  if (stride != 1 || in_ch != out_ch) {
    sc.push_back(std::make_unique<Conv2D>(in_ch, out_ch, 1, 1, stride, stride, 0, 0, false, "conv2d_0"));
    sc.push_back(std::make_unique<BatchNorm>(out_ch, 1e-3f, 0.1f, true, "bn0"));
  }
  return residual(std::move(m), std::move(sc), "relu",
                  name.empty() ? "bottleneck_residual_block_" + std::to_string(model_.layers().size()) : name);
}

Sequential SequentialBuilder::build() { return std::move(model_); }

// ------------------------------------------------------------------ loss
LossResult softmax_cross_entropy(const Tensor& logits, const Tensor& labels_in) {
  if (logits.rank() != 2) throw std::runtime_error("softmax_cross_entropy: expected [N, C] logits");
  const int N = (int)logits.dim(0), C = (int)logits.dim(1);
  const Device dev = logits.device();
  Tensor labels = labels_in.device() == dev ? labels_in : labels_in.to(dev);
  LossResult r;
  if (dev.is_gpu()) {
    r.grad = Tensor::empty({N, C}, DType::BF16, dev, Layout::NHWC);
    r.loss = gpu_ops::softmax_ce(logits.data(), labels.ptr<int64_t>(), r.grad.data(), N, C, &r.correct);
  } else {
    r.grad = Tensor::empty({N, C}, DType::F32, dev);
    r.loss = cpu_ops::softmax_ce(logits.ptr<float>(), labels.ptr<int64_t>(), r.grad.ptr<float>(), N, C, &r.correct);
  }
  return r;
}

// ------------------------------------------------------------------ optimizers
namespace {
// every parameter of one arena, and nothing else: one fused update over the flat buffers
ParamArena* whole_arena(const std::vector<Param*>& params) {
  if (params.empty() || !params[0]->arena || params[0]->arena->count != params.size()) return nullptr;
  ParamArena* a = params[0]->arena.get();
  for (auto* p : params)
    if (p->arena.get() != a) return nullptr;
  return a;
}
}  // namespace

void SGD::step(const std::vector<Param*>& params) {
  if (ParamArena* a = whole_arena(params)) {
    gpu_ops::sgd(a->value.ptr<float>(), a->grad.ptr<float>(), momentum_ != 0.f ? a->m.ptr<float>() : nullptr,
                 a->shadow.data(), (long)a->n, lr_, momentum_);
    a->refresh_transposes();
    return;
  }
  for (auto* p : params) {
    if (p->arena) p->arena->wt_valid = false;  // (the convs transpose their own operand)
    if (momentum_ != 0.f && !p->m.defined()) p->m = Tensor::zeros(p->value.shape(), DType::F32, p->value.device());
    float* vel = momentum_ != 0.f ? p->m.ptr<float>() : nullptr;
    if (p->value.device().is_gpu())
      gpu_ops::sgd(p->value.ptr<float>(), p->grad.ptr<float>(), vel, p->shadow.data(), p->value.numel(), lr_,
                   momentum_);
    else
      cpu_ops::sgd(p->value.ptr<float>(), p->grad.ptr<float>(), vel, p->value.numel(), lr_, momentum_);
  }
}

void Adam::upload_hyper() {
  if (!hyper_.defined()) return;
  const float h[4] = {lr_, 0.f, 0.f, (float)t_};  // bc1 / bc2 are recomputed by the next step
  gpu::copy(hyper_.data(), h, sizeof h, 0);
  hyper_lr_ = lr_;
  hyper_t_ = t_;
}

void Adam::before_replay() {
  if (hyper_.defined() && hyper_lr_ != lr_) {
    gpu::copy(hyper_.data(), &lr_, sizeof lr_, 0);
    hyper_lr_ = lr_;
  }
  ++t_;
  ++hyper_t_;
}

void Adam::step(const std::vector<Param*>& params) {
  if (ParamArena* a = whole_arena(params)) {
    // step scalars on the device (a captured step replays with the current lr and t)
    if (!hyper_.defined()) hyper_ = Tensor::zeros({4}, DType::F32, a->value.device());
    if (hyper_lr_ != lr_ || hyper_t_ != t_) {
      if (gpu::Graph::capturing()) throw std::runtime_error("Adam: step scalars changed inside a graph capture");
      upload_hyper();
    }
    ++t_;
    ++hyper_t_;
    gpu_ops::adam_hyper_step(hyper_.ptr<float>(), b1_, b2_);
    gpu_ops::adam_dev(a->value.ptr<float>(), a->grad.ptr<float>(), a->m.ptr<float>(), a->v.ptr<float>(),
                      a->shadow.data(), (long)a->n, b1_, b2_, eps_, wd_, decoupled_, hyper_.ptr<float>());
    a->refresh_transposes();
    return;
  }
  ++t_;
  const float bc1 = 1.f - std::pow(b1_, (float)t_), bc2 = 1.f - std::pow(b2_, (float)t_);
  for (auto* p : params) {
    if (p->arena) p->arena->wt_valid = false;
    if (!p->m.defined()) {
      p->m = Tensor::zeros(p->value.shape(), DType::F32, p->value.device());
      p->v = Tensor::zeros(p->value.shape(), DType::F32, p->value.device());
    }
    if (p->value.device().is_gpu())
      gpu_ops::adam(p->value.ptr<float>(), p->grad.ptr<float>(), p->m.ptr<float>(), p->v.ptr<float>(),
                    p->shadow.data(), p->value.numel(), lr_, b1_, b2_, eps_, bc1, bc2, wd_, decoupled_);
    else
      cpu_ops::adam(p->value.ptr<float>(), p->grad.ptr<float>(), p->m.ptr<float>(), p->v.ptr<float>(),
                    p->value.numel(), lr_, b1_, b2_, eps_, bc1, bc2, wd_, decoupled_);
  }
}

// ------------------------------------------------------------------ data
SyntheticClassification::SyntheticClassification(size_t n, int c, int h, int w, int classes, uint64_t seed,
                                                 float noise)
    : n_(n), c_(c), h_(h), w_(w), classes_(classes), seed_(seed), noise_(noise) {
  Rng r(seed ^ 0x5151u);
  proto_.resize((size_t)classes * c * h * w);
  for (auto& v : proto_) v = r.normal();
  order_.resize(n);
  for (size_t i = 0; i < n; ++i) order_[i] = i;
}

void SyntheticClassification::reset(uint64_t epoch) {
  Rng r(seed_ + 977 * (epoch + 1));
  for (size_t i = n_; i > 1; --i) std::swap(order_[i - 1], order_[(size_t)(r.next() % i)]);
  pos_ = 0;
}

bool SyntheticClassification::next(int batch, Tensor& x, Tensor& labels) {
  if (pos_ >= n_) return false;
  const int b = (int)std::min<size_t>((size_t)batch, n_ - pos_);
  const size_t per = (size_t)c_ * h_ * w_;
  std::vector<float> xs((size_t)b * per);
  std::vector<int64_t> ys((size_t)b);
  for (int i = 0; i < b; ++i) {
    const size_t idx = order_[pos_ + i];
    Rng r(seed_ * 1315423911ull + idx);
    const int cls = (int)(idx % (size_t)classes_);
    ys[i] = cls;
    const float* pr = proto_.data() + (size_t)cls * per;
    for (size_t k = 0; k < per; ++k) xs[i * per + k] = pr[k] + noise_ * r.normal();
  }
  pos_ += (size_t)b;
  x = Tensor::from_host(xs, {b, c_, h_, w_}, Device::cpu());
  labels = Tensor::from_host_i64(ys, Device::cpu());
  return true;
}

// ------------------------------------------------------------------ training loop
LossResult train_step(Sequential& model, Optimizer& opt, const Tensor& x, const Tensor& labels) {
  model.set_training(true);
  model.zero_grad();
  Tensor logits = model.forward(x);
  LossResult r = softmax_cross_entropy(logits, labels);
  model.backward(r.grad);
  opt.step(model.parameters());
  return r;
}

EpochStats evaluate(Sequential& model, DataSource& src, int batch_size) {
  const bool was = model.is_training();
  model.set_training(false);
  src.reset(0);
  Tensor x, y;
  double loss = 0;
  long correct = 0, seen = 0;
  while (src.next(batch_size, x, y)) {
    Tensor logits = model.forward(x);
    LossResult r = softmax_cross_entropy(logits, y);
    loss += r.loss * x.dim(0);
    correct += r.correct;
    seen += x.dim(0);
  }
  model.set_training(was);
  EpochStats s;
  s.val_loss = seen ? loss / seen : 0;
  s.val_acc = seen ? (double)correct / seen : 0;
  return s;
}

std::vector<EpochStats> train_classification_model(Sequential& model, DataSource& train, DataSource* val,
                                                   Optimizer& opt, const TrainingConfig& cfg) {
  std::vector<EpochStats> hist;
  for (int e = 0; e < cfg.epochs; ++e) {
    const auto t0 = std::chrono::steady_clock::now();
    train.reset(cfg.seed + (uint64_t)e);
    Tensor x, y;
    double loss = 0;
    long correct = 0, seen = 0;
    int step = 0;
    while ((cfg.max_steps < 0 || step < cfg.max_steps) && train.next(cfg.batch_size, x, y)) {
      LossResult r = train_step(model, opt, x, y);
      loss += r.loss * x.dim(0);
      correct += r.correct;
      seen += x.dim(0);
      ++step;
      if (cfg.progress_interval > 0 && step % cfg.progress_interval == 0)
        std::printf("epoch %d step %d  loss %.4f  acc %.2f%%\n", e + 1, step, loss / seen, 100.0 * correct / seen);
    }
    EpochStats s;
    s.train_loss = seen ? loss / seen : 0;
    s.train_acc = seen ? (double)correct / seen : 0;
    if (val) {
      EpochStats v = evaluate(model, *val, cfg.batch_size);
      s.val_loss = v.val_loss;
      s.val_acc = v.val_acc;
    }
    if (model.device().is_gpu()) gpu::synchronize();
    s.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("epoch %d/%d  train loss %.4f acc %.2f%%  val loss %.4f acc %.2f%%  (%.2f s)\n", e + 1, cfg.epochs,
                s.train_loss, 100 * s.train_acc, s.val_loss, 100 * s.val_acc, s.seconds);
    hist.push_back(s);
    opt.set_learning_rate(opt.learning_rate() * cfg.lr_decay);
  }
  return hist;
}

}  // namespace dcnn
