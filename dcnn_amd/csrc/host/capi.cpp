// C ABI over the C++ host API's GPU convolution entry points (dcnn/ops.hpp gpu_ops), for tests that
// drive the C++ engine's own plumbing from Python (ctypes on libdcnn.so, device pointers of torch
// tensors): tests/test_gpu_cpp_geometry.py replays every conv call a production C++ training step
// records (DCNN_RECORD_OPS) through these functions and compares with fp32 PyTorch.
//
// Every call runs on the calling thread's flow and synchronises the device before it returns (the
// caller synchronises its own stream before the call). Returns 0, or -1 with dcnn_c_last_error().
// shape[13] = ConvShape {N, C, H, W, Co, KH, KW, SH, SW, PH, PW, OH, OW}.
// Reference parity: unit_tests/conv2d_layer_test.cpp:660-990 drives the reference's conv layer the
// same way (per-shape calls against a loop reference).
#include <cstring>
#include <exception>
#include <string>

#include "dcnn/ops.hpp"
#include "dcnn/tensor.hpp"

using namespace dcnn;

namespace {
thread_local std::string t_err;

ConvShape shape_of(const int* v) {
  return ConvShape{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12]};
}

template <typename F>
int guarded(F&& f) {
  try {
    f();
    gpu::synchronize();
    return 0;
  } catch (const std::exception& e) {
    t_err = e.what();
  } catch (...) {
    t_err = "unknown error";
  }
  return -1;
}
}  // namespace

extern "C" {

const char* dcnn_c_last_error() { return t_err.c_str(); }

void dcnn_c_set_fault(int f) { gpu_ops::set_fault(f); }

int dcnn_c_copy(void* dst, const void* src, size_t nbytes) {
  return guarded([&] { gpu::copy(dst, src, nbytes, 2); });
}

// y = conv(x, w) + bias; want_stats: *slab / *rows = the epilogue's [rows][3][Co] Welford rows
int dcnn_c_conv_fwd(const void* x, const void* w, const float* bias, void* y, const int* shape, int want_stats,
                    const float** slab, int* rows) {
  return guarded([&] {
    int r = 0;
    const float* s = gpu_ops::conv_fwd(x, w, bias, y, shape_of(shape), want_stats ? &r : nullptr);
    if (slab) *slab = s;
    if (rows) *rows = r;
  });
}

// dx = dgrad(dy, w) (+ residual); w_t: w is transposed here first and passed as the pre-transposed
// operand (the arena path); bnb: the fused BatchNorm backward (mask y_bn when non-null, statistics
// rows [rows][2][C] in *slab)
int dcnn_c_conv_dgrad(const void* dy, const void* w, int w_t, void* dx, const int* shape, const void* residual,
                      int bnb, const void* y_bn, const void* x_bn, const float* mean, const float* istd,
                      const float** slab, int* rows) {
  return guarded([&] {
    const ConvShape s = shape_of(shape);
    Tensor wt;
    const void* wop = w;
    if (w_t) {
      int dev = 0;
      wt = Tensor::empty({(int64_t)s.C * s.KH * s.KW * s.Co}, DType::BF16, Device::gpu(dev));
      gpu_ops::weight_transpose(w, wt.data(), s.Co, s.KH * s.KW, s.C);
      wop = wt.data();
    }
    gpu_ops::BnbOperands ops{y_bn, x_bn, mean, istd};
    int r = 0;
    const float* st = gpu_ops::conv_dgrad(dy, wop, dx, s, residual, w_t != 0, bnb ? &ops : nullptr, &r);
    if (slab) *slab = st;
    if (rows) *rows = r;
    gpu::synchronize();  // (wt is released after the kernels that read it)
  });
}

// gw / gb (+=) the weight / bias gradient; deferred: inside a backward's batched split-K reduce
int dcnn_c_conv_wgrad(const void* dy, const void* x, float* gw, float* gb, const int* shape, int deferred) {
  return guarded([&] {
    if (deferred) gpu_ops::begin_deferred_reduce();
    try {
      gpu_ops::conv_wgrad(dy, x, gw, gb, shape_of(shape));
    } catch (...) {
      if (deferred) gpu_ops::end_deferred_reduce();
      throw;
    }
    if (deferred) gpu_ops::end_deferred_reduce();
  });
}

int dcnn_c_stem_fwd(const float* x, const void* w, const float* bias, void* y, const int* shape, int want_stats,
                    const float** slab, int* rows) {
  return guarded([&] {
    int r = 0;
    const float* s = gpu_ops::stem_fwd(x, w, bias, y, shape_of(shape), want_stats ? &r : nullptr);
    if (slab) *slab = s;
    if (rows) *rows = r;
  });
}

int dcnn_c_stem_wgrad(const void* dy, const float* x, float* gw, float* gb, const int* shape, int deferred) {
  return guarded([&] {
    if (deferred) gpu_ops::begin_deferred_reduce();
    try {
      gpu_ops::stem_wgrad(dy, x, gw, gb, shape_of(shape));
    } catch (...) {
      if (deferred) gpu_ops::end_deferred_reduce();
      throw;
    }
    if (deferred) gpu_ops::end_deferred_reduce();
  });
}

}  // extern "C"
