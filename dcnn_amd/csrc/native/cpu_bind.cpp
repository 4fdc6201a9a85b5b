// pybind11 surface of the native CPU backend (`_native.cpu`): raw host pointers from
// torch.Tensor.data_ptr() plus a dtype code (0 = float32, 1 = float64); the Python side
// (dcnn_amd/ops/cpu.py) checks shapes, contiguity and dtypes before calling in. Long-running
// calls release the GIL so pipeline stage threads and data loaders keep running.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <utility>

#include "cpu_kernels.h"
#include "threadpool.h"

namespace py = pybind11;
using namespace dcnn_native;
using namespace dcnn_native::cpu;

namespace {
template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
#define DT_DISPATCH(dt, CALL)                                   \
  do {                                                          \
    if ((dt) == 0) {                                            \
      using T = float;                                          \
      CALL;                                                     \
    } else if ((dt) == 1) {                                     \
      using T = double;                                         \
      CALL;                                                     \
    } else {                                                    \
      throw std::invalid_argument("cpu backend: dtype code must be 0 (f32) or 1 (f64)"); \
    }                                                           \
  } while (0)
using Rel = py::call_guard<py::gil_scoped_release>;
}  // namespace

void bind_cpu(py::module_& parent) {
  py::module_ m = parent.def_submodule("cpu", "native CPU compute backend (float32 / float64, NCHW)");
  m.def("set_num_threads", &set_num_threads);
  m.def("get_num_threads", &get_num_threads);
  m.def("gemm_uses_avx2", &gemm_uses_avx2);
  m.def("gemm_uses_avx512", &gemm_uses_avx512);
  m.def("gemm", [](int dt, bool ta, bool tb, long M, long N, long K, double alpha, uintptr_t A, long lda, uintptr_t B,
                   long ldb, double beta, uintptr_t C, long ldc) {
    DT_DISPATCH(dt, gemm(ta, tb, M, N, K, (T)alpha, P<const T>(A), lda, P<const T>(B), ldb, (T)beta, P<T>(C), ldc));
  }, Rel());
  m.def("elementwise", [](int dt, int mode, int op, uintptr_t a, uintptr_t b, uintptr_t c, long n, double s0,
                          double s1) {
    DT_DISPATCH(dt, elementwise<T>(mode, op, P<const T>(a), P<const T>(b), P<T>(c), n, s0, s1));
  }, Rel());
  m.def("reduce", [](int dt, int op, uintptr_t a, uintptr_t b, long n) {
    double r = 0;
    DT_DISPATCH(dt, r = reduce<T>(op, P<const T>(a), P<const T>(b), n));
    return r;
  }, Rel());
  m.def("fill_random", [](int dt, uintptr_t out, long n, uint64_t seed, double a, double b, int normal) {
    DT_DISPATCH(dt, fill_random<T>(P<T>(out), n, seed, a, b, normal));
  }, Rel());
  m.def("transpose2d", [](int dt, uintptr_t in, uintptr_t out, long batch, long rows, long cols) {
    DT_DISPATCH(dt, transpose2d<T>(P<const T>(in), P<T>(out), batch, rows, cols));
  }, Rel());
  m.def("swap01", [](int dt, uintptr_t in, uintptr_t out, long A, long B, long HW) {
    DT_DISPATCH(dt, swap01<T>(P<const T>(in), P<T>(out), A, B, HW));
  }, Rel());
  m.def("pad2d", [](int dt, uintptr_t x, uintptr_t y, long NC, int H, int W, int ph, int pw, double v) {
    DT_DISPATCH(dt, pad2d<T>(P<const T>(x), P<T>(y), NC, H, W, ph, pw, v));
  }, Rel());
  m.def("crop2d", [](int dt, uintptr_t x, uintptr_t y, long NC, int H, int W, int top, int left, int OH, int OW) {
    DT_DISPATCH(dt, crop2d<T>(P<const T>(x), P<T>(y), NC, H, W, top, left, OH, OW));
  }, Rel());
  m.def("im2col", [](int dt, uintptr_t x, uintptr_t col, int N, int C, int H, int W, int KH, int KW, int SH, int SW,
                     int PH, int PW) {
    DT_DISPATCH(dt, im2col<T>(P<const T>(x), P<T>(col), N, C, H, W, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("col2im", [](int dt, uintptr_t col, uintptr_t x, int N, int C, int H, int W, int KH, int KW, int SH, int SW,
                     int PH, int PW) {
    DT_DISPATCH(dt, col2im<T>(P<const T>(col), P<T>(x), N, C, H, W, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("conv2d_fwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int C, int H, int W,
                         int Co, int KH, int KW, int SH, int SW, int PH, int PW) {
    DT_DISPATCH(dt, conv2d_fwd<T>(P<const T>(x), P<const T>(w), P<const T>(bias), P<T>(y), N, C, H, W, Co, KH, KW, SH,
                                  SW, PH, PW));
  }, Rel());
  m.def("conv2d_bwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t dy, uintptr_t dx, uintptr_t dw, uintptr_t db,
                         int N, int C, int H, int W, int Co, int KH, int KW, int SH, int SW, int PH, int PW) {
    DT_DISPATCH(dt, conv2d_bwd<T>(P<const T>(x), P<const T>(w), P<const T>(dy), P<T>(dx), P<T>(dw), P<T>(db), N, C, H,
                                  W, Co, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("dense_fwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, long N, long In, long Out) {
    DT_DISPATCH(dt, dense_fwd<T>(P<const T>(x), P<const T>(w), P<const T>(bias), P<T>(y), N, In, Out));
  }, Rel());
  m.def("dense_bwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t dy, uintptr_t dx, uintptr_t dw, uintptr_t db,
                        long N, long In, long Out) {
    DT_DISPATCH(dt, dense_bwd<T>(P<const T>(x), P<const T>(w), P<const T>(dy), P<T>(dx), P<T>(dw), P<T>(db), N, In,
                                 Out));
  }, Rel());
  m.def("batchnorm_fwd", [](int dt, uintptr_t x, uintptr_t y, long N, long C, long HW, uintptr_t gamma,
                            uintptr_t beta, double eps, int training, uintptr_t rmean, uintptr_t rvar, double momentum,
                            uintptr_t smean, uintptr_t sistd, int relu, uintptr_t residual) {
    DT_DISPATCH(dt, batchnorm_fwd<T>(P<const T>(x), P<T>(y), N, C, HW, P<const T>(gamma), P<const T>(beta), eps,
                                     training, P<T>(rmean), P<T>(rvar), momentum, P<T>(smean), P<T>(sistd), relu,
                                     P<const T>(residual)));
  }, Rel());
  m.def("batchnorm_bwd", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t yout, uintptr_t mean, uintptr_t istd,
                            uintptr_t gamma, uintptr_t dx, uintptr_t dgamma, uintptr_t dbeta, uintptr_t masked, long N,
                            long C, long HW, int training) {
    DT_DISPATCH(dt, batchnorm_bwd<T>(P<const T>(x), P<const T>(dy), P<const T>(yout), P<const T>(mean),
                                     P<const T>(istd), P<const T>(gamma), P<T>(dx), P<T>(dgamma), P<T>(dbeta),
                                     P<T>(masked), N, C, HW, training));
  }, Rel());
  m.def("groupnorm_fwd", [](int dt, uintptr_t x, uintptr_t y, long N, long C, long HW, long G, uintptr_t gamma,
                            uintptr_t beta, double eps, uintptr_t smean, uintptr_t sistd) {
    DT_DISPATCH(dt, groupnorm_fwd<T>(P<const T>(x), P<T>(y), N, C, HW, G, P<const T>(gamma), P<const T>(beta), eps,
                                     P<T>(smean), P<T>(sistd)));
  }, Rel());
  m.def("groupnorm_bwd", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t mean, uintptr_t istd, uintptr_t gamma,
                            uintptr_t dx, uintptr_t dgamma, uintptr_t dbeta, long N, long C, long HW, long G) {
    DT_DISPATCH(dt, groupnorm_bwd<T>(P<const T>(x), P<const T>(dy), P<const T>(mean), P<const T>(istd),
                                     P<const T>(gamma), P<T>(dx), P<T>(dgamma), P<T>(dbeta), N, C, HW, G));
  }, Rel());
  m.def("maxpool_fwd", [](int dt, uintptr_t x, uintptr_t y, uintptr_t idx, long NC, int H, int W, int KH, int KW,
                          int SH, int SW, int PH, int PW) {
    DT_DISPATCH(dt, maxpool_fwd<T>(P<const T>(x), P<T>(y), P<int32_t>(idx), NC, H, W, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("maxpool_bwd", [](int dt, uintptr_t dy, uintptr_t idx, uintptr_t dx, long NC, int H, int W, int OH, int OW) {
    DT_DISPATCH(dt, maxpool_bwd<T>(P<const T>(dy), P<const int32_t>(idx), P<T>(dx), NC, H, W, OH, OW));
  }, Rel());
  m.def("avgpool_fwd", [](int dt, uintptr_t x, uintptr_t y, long NC, int H, int W, int KH, int KW, int SH, int SW,
                          int PH, int PW) {
    DT_DISPATCH(dt, avgpool_fwd<T>(P<const T>(x), P<T>(y), NC, H, W, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("avgpool_bwd", [](int dt, uintptr_t dy, uintptr_t dx, long NC, int H, int W, int KH, int KW, int SH, int SW,
                          int PH, int PW) {
    DT_DISPATCH(dt, avgpool_bwd<T>(P<const T>(dy), P<T>(dx), NC, H, W, KH, KW, SH, SW, PH, PW));
  }, Rel());
  m.def("act_fwd", [](int dt, int type, uintptr_t x, uintptr_t y, long n, double alpha) {
    DT_DISPATCH(dt, act_fwd<T>(type, P<const T>(x), P<T>(y), n, alpha));
  }, Rel());
  m.def("act_bwd", [](int dt, int type, uintptr_t x, uintptr_t dy, uintptr_t dx, long n, double alpha) {
    DT_DISPATCH(dt, act_bwd<T>(type, P<const T>(x), P<const T>(dy), P<T>(dx), n, alpha));
  }, Rel());
  m.def("softmax_channels", [](int dt, uintptr_t x, uintptr_t y, long N, long C, long HW) {
    DT_DISPATCH(dt, softmax_channels<T>(P<const T>(x), P<T>(y), N, C, HW));
  }, Rel());
  m.def("softmax_channels_bwd", [](int dt, uintptr_t y, uintptr_t dy, uintptr_t dx, long N, long C, long HW) {
    DT_DISPATCH(dt, softmax_channels_bwd<T>(P<const T>(y), P<const T>(dy), P<T>(dx), N, C, HW));
  }, Rel());
  m.def("loss_fused", [](int dt, int kind, uintptr_t pred, uintptr_t target, uintptr_t labels, uintptr_t grad, long N,
                         long C, double param) {
    double l = 0;
    long correct = 0;
    DT_DISPATCH(dt, l = loss_fused<T>(kind, P<const T>(pred), P<const T>(target), P<const int64_t>(labels), P<T>(grad),
                                      N, C, param, &correct));
    return std::make_pair(l, correct);  // converted after the GIL is re-acquired
  }, Rel());
  m.def("sgd_step", [](int dt, uintptr_t p, uintptr_t g, uintptr_t vel, long n, double lr, double mom) {
    DT_DISPATCH(dt, sgd_step<T>(P<T>(p), P<const T>(g), P<T>(vel), n, lr, mom));
  }, Rel());
  m.def("adam_step", [](int dt, uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, long n, double lr, double b1,
                        double b2, double eps, double bc1, double bc2, double wd, int dec) {
    DT_DISPATCH(dt, adam_step<T>(P<T>(p), P<const T>(g), P<T>(mm), P<T>(v), n, lr, b1, b2, eps, bc1, bc2, wd, dec));
  }, Rel());
}
