// pybind11 entry points of the HIP kernel library. Arguments are raw device pointers
// (uintptr_t, from torch.Tensor.data_ptr()) and the hipStream_t of the caller's current
// stream, so launches land on whatever stream PyTorch-ROCm is using (including a stream
// under hipGraph capture). No torch headers, no hipify: plain HIP + pybind11.
#include <tuple>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <algorithm>
#include <array>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace py = pybind11;
#include "api.h"


using namespace dcnn;
void bind_runtime(py::module_& m);  // runtime.cpp: native Device / Flow / Task / Allocator
void bind_rccl(py::module_& m);     // rccl.cpp: in-tree RCCL communicator (dlopen)
template <typename T>
static inline T P(uintptr_t x) { return reinterpret_cast<T>(x); }
static inline hipStream_t S(uintptr_t x) { return reinterpret_cast<hipStream_t>(x); }

static void bind_gemm_g2(uintptr_t A, uintptr_t B, uintptr_t C, unsigned a_bytes, unsigned b_bytes, int M, int N, int Cs,
                         int H, int W, int GH, int GW, int SY, int SX, std::vector<std::array<int, 4>> taps, int ldb,
                         int ldc, int OH, int OW, int OSY, int OSX, int ORY, int ORX, uintptr_t bias, uintptr_t residual,
                         uintptr_t stats, int relu, uintptr_t zero_ptr, int zero_n, std::array<uintptr_t, 4> bnb,
                         uintptr_t stream, std::vector<std::array<int, 4>> classes = {}) {
  G2Args a{};
  // classes: (first tap, taps, ORY, ORX) per row class of a grouped launch (empty: one class)
  if (classes.size() > 4) throw std::runtime_error("gemm_g2: at most 4 row classes");
  a.ncls = (int)classes.size();
  a.cls_rows = classes.empty() ? 0 : M / (int)classes.size();
  for (size_t c = 0; c < classes.size(); ++c) {
    a.cls_t0[c] = classes[c][0]; a.cls_nt[c] = classes[c][1]; a.cls_ory[c] = classes[c][2]; a.cls_orx[c] = classes[c][3];
  }
  a.bnb = BnbArgs{P<const bf16*>(bnb[0]), P<const bf16*>(bnb[1]), P<const float*>(bnb[2]), P<const float*>(bnb[3])};
  a.A = P<const bf16*>(A); a.B = P<const bf16*>(B); a.C = P<bf16*>(C);
  a.a_bytes = a_bytes; a.b_bytes = b_bytes;
  a.M = M; a.N = N; a.Cs = Cs; a.H = H; a.W = W; a.GH = GH; a.GW = GW; a.SY = SY; a.SX = SX;
  if (taps.size() > 64) throw std::runtime_error("gemm_g2: more than 64 taps");
  a.ntaps = (int)taps.size();
  for (size_t i = 0; i < taps.size(); ++i) {
    a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; a.tap_srcoff[i] = taps[i][2]; a.tap_b[i] = taps[i][3];
  }
  a.ldb = ldb; a.ldc = ldc; a.OH = OH; a.OW = OW; a.OSY = OSY; a.OSX = OSX; a.ORY = ORY; a.ORX = ORX;
  a.bias = P<const float*>(bias); a.residual = P<const bf16*>(residual); a.stats = P<float*>(stats); a.relu = relu;
  a.zero_ptr = P<float*>(zero_ptr); a.zero_n = zero_n;
  gemm_g2(a, S(stream));
}

PYBIND11_MODULE(_kernels, m) {
  m.doc() = "dcnn_amd HIP/CDNA4 (gfx950) kernel library";
  m.attr("arch") = "gfx950";
  bind_runtime(m);
  bind_rccl(m);

  m.def("gemm_nt",
        [](uintptr_t A, uintptr_t B, uintptr_t C, int M, int N, int K, int lda, int ldb, int ldc, int mode, int nb,
           int sh, int sw, int cs, int gh, int gw, int kh, int kw, int strh, int strw, int padh, int padw,
           uintptr_t bias, uintptr_t residual, uintptr_t stats, int out_f32, int relu, uintptr_t stream) {
          NtArgs a{P<const bf16*>(A), P<const bf16*>(B), P<void*>(C), M, N, K, lda, ldb, ldc, mode, nb, sh, sw, cs, gh,
                   gw, kh, kw, strh, strw, padh, padw, P<const float*>(bias), P<const bf16*>(residual),
                   P<float*>(stats), out_f32, relu};
          gemm_nt(a, S(stream));
        });
  m.def("gemm_nt_stat_rows", &gemm_nt_stat_rows);
  m.def("elementwise", [](int mode, int op, uintptr_t a, uintptr_t b, uintptr_t c, long n, float s0, float s1,
                          uintptr_t st) {
    elementwise(mode, op, P<const float*>(a), P<const float*>(b), P<float*>(c), n, s0, s1, S(st));
  });
  m.def("reduce", [](int op, uintptr_t a, uintptr_t b, long n, uintptr_t ws, uintptr_t out, uintptr_t st) {
    reduce(op, P<const float*>(a), P<const float*>(b), n, P<float*>(ws), P<float*>(out), S(st));
  });
  m.def("fill_random", [](uintptr_t out, long n, uint64_t seed, float a, float b, int normal, uintptr_t st) {
    fill_random(P<float*>(out), n, seed, a, b, normal, S(st));
  });
  m.def("transpose_batched16", [](uintptr_t in, uintptr_t out, int batch, int rows, int cols, uintptr_t st) {
    transpose_batched16(P<const void*>(in), P<void*>(out), batch, rows, cols, S(st));
  });
  m.def("rows_copy", [](int kind, uintptr_t src, int lds, uintptr_t dst, int ldd, long rows, int cols, uintptr_t st) {
    rows_copy(kind, P<const void*>(src), lds, P<void*>(dst), ldd, rows, cols, S(st));
  });
  m.def("transpose_batched", [](uintptr_t in, uintptr_t out, int batch, int rows, int cols, uintptr_t st) {
    transpose_batched(P<const float*>(in), P<float*>(out), batch, rows, cols, S(st));
  });
  m.def("nchw_cnhw", [](uintptr_t in, uintptr_t out, int N, int C, int HW, int to_cnhw, uintptr_t st) {
    nchw_cnhw(P<const float*>(in), P<float*>(out), N, C, HW, to_cnhw, S(st));
  });
  m.def("pad_crop", [](uintptr_t in, uintptr_t out, int NC, int H, int W, int OH, int OW, int top, int left,
                       float value, uintptr_t st) {
    pad_crop(P<const float*>(in), P<float*>(out), NC, H, W, OH, OW, top, left, value, S(st));
  });
  m.def("hconv",
        [](uintptr_t A, uintptr_t B, uintptr_t C, unsigned a_bytes, unsigned b_bytes, int NB, int H, int W, int Cs,
           int N, int ldb, std::vector<std::array<int, 3>> taps, uintptr_t bias, uintptr_t residual, uintptr_t stats,
           int relu, uintptr_t zero_ptr, int zero_n, std::array<uintptr_t, 4> bnb, uintptr_t Cf, uintptr_t residual_f,
           int splits, uintptr_t part, uintptr_t tickets, uintptr_t stream) {
          HConvArgs a{};
          a.splits = splits; a.part = P<float*>(part); a.tickets = P<unsigned*>(tickets);
          a.Cf = P<float*>(Cf); a.residual_f = P<const float*>(residual_f);
          a.bnb = BnbArgs{P<const bf16*>(bnb[0]), P<const bf16*>(bnb[1]), P<const float*>(bnb[2]), P<const float*>(bnb[3])};
          a.zero_ptr = P<float*>(zero_ptr); a.zero_n = zero_n;
          a.A = P<const bf16*>(A); a.B = P<const bf16*>(B); a.C = P<bf16*>(C);
          a.a_bytes = a_bytes; a.b_bytes = b_bytes;
          a.NB = NB; a.H = H; a.W = W; a.Cs = Cs; a.N = N; a.ldb = ldb;
          if (taps.size() > 9 || taps.empty()) throw std::runtime_error("hconv: 1..9 taps");
          a.ntaps = (int)taps.size();
          for (size_t i = 0; i < taps.size(); ++i) { a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; a.tap_b[i] = taps[i][2]; }
          a.bias = P<const float*>(bias); a.residual = P<const bf16*>(residual); a.stats = P<float*>(stats); a.relu = relu;
          hconv(a, S(stream));
        });
  m.def("hconv3_f32",
        [](uintptr_t A, uintptr_t B, unsigned a_bytes, unsigned b_bytes, int NB, int H, int W, int Cs, int N, int ldb,
           std::vector<std::array<int, 3>> taps, uintptr_t bias, uintptr_t stats, int relu, uintptr_t zero_ptr,
           int zero_n, uintptr_t Cf, uintptr_t residual_f, int splits, uintptr_t part, uintptr_t tickets,
           uintptr_t stream, std::array<uintptr_t, 4> bnb) {
          HConvArgs a{};
          // backward-BatchNorm fusion: (y, x, mean, istd), y / x the BatchNorm's fp32 tensors
          a.bnb.y = P<const bf16*>(bnb[0]); a.bnb.x = P<const bf16*>(bnb[1]);
          a.bnb.mean = P<const float*>(bnb[2]); a.bnb.istd = P<const float*>(bnb[3]);
          a.splits = splits; a.part = P<float*>(part); a.tickets = P<unsigned*>(tickets);
          a.Cf = P<float*>(Cf); a.residual_f = P<const float*>(residual_f);
          a.zero_ptr = P<float*>(zero_ptr); a.zero_n = zero_n;
          a.A = P<const bf16*>(A); a.B = P<const bf16*>(B);
          a.a_bytes = a_bytes; a.b_bytes = b_bytes;
          a.NB = NB; a.H = H; a.W = W; a.Cs = Cs; a.N = N; a.ldb = ldb;
          if (taps.size() != 9) return false;
          a.ntaps = 9;
          for (size_t i = 0; i < taps.size(); ++i) { a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; a.tap_b[i] = taps[i][2]; }
          a.bias = P<const float*>(bias); a.stats = P<float*>(stats); a.relu = relu;
          return hconv3_f32_try(a, S(stream));
        },
        py::arg("A"), py::arg("B"), py::arg("a_bytes"), py::arg("b_bytes"), py::arg("NB"), py::arg("H"), py::arg("W"),
        py::arg("Cs"), py::arg("N"), py::arg("ldb"), py::arg("taps"), py::arg("bias"), py::arg("stats"),
        py::arg("relu"), py::arg("zero_ptr"), py::arg("zero_n"), py::arg("Cf"), py::arg("residual_f"),
        py::arg("splits"), py::arg("part"), py::arg("tickets"), py::arg("stream"),
        py::arg("bnb") = std::array<uintptr_t, 4>{0, 0, 0, 0});
  m.def("hconv3_f32_splits", &hconv3_f32_splits);
  m.def("hconv_supported", &hconv_supported);
  m.def("hconv_stat_rows", &hconv_stat_rows);
  m.def("hconv_splits", &hconv_splits);
  m.def("hconv_tiles", &hconv_tiles);
  m.def("hconv_set_split_target", &hconv_set_split_target);
  m.def("hconv_set_split_min_work", &hconv_set_split_min_work);
  m.def("hconv_split_target", &hconv_split_target);
  m.def("gemm_t2_set_split_target", &gemm_t2_set_split_target);
  m.def("hwgrad_set_split_target", &hwgrad_set_split_target);
  m.def("hconv3_set_max_splits", &hconv3_set_max_splits);
  m.def("bn_set_vectorised", &bn_set_vectorised);
  m.def("hconv_tile_elems", &hconv_tile_elems);
  m.def("hconv3_set_grid_cap", &hconv3_set_grid_cap);
  m.def("hconv3_enable", &hconv3_enable);
  m.def("hconv_v3", &hconv_v3);
  m.def("hconv3_set_stamps", &hconv3_set_stamps);
  m.def("hwgrad",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, unsigned dy_bytes, unsigned x_bytes, int NB,
           int H, int W, int Cs, int Co, std::vector<std::array<int, 2>> taps, int splits, int ldy, int ldx,
           std::vector<std::array<int, 3>> pairs, uintptr_t stream) {
          HWArgs a{};
          if (pairs.size() > 3) throw std::runtime_error("hwgrad: at most 3 operand pairs");
          a.npairs = (int)pairs.size(); a.ldy = ldy; a.ldx = ldx;  // no pairs: the plain wgrad
          for (size_t q = 0; q < pairs.size(); ++q) {
            a.pair_yoff[q] = pairs[q][0]; a.pair_xoff[q] = pairs[q][1]; a.pair_bias[q] = pairs[q][2];
          }
          a.dY = P<const bf16*>(dY); a.X = P<const bf16*>(X); a.slab = P<float*>(slab);
          a.bias_slab = P<float*>(bias_slab);
          a.dy_bytes = dy_bytes; a.x_bytes = x_bytes;
          a.NB = NB; a.H = H; a.W = W; a.Cs = Cs; a.Co = Co;
          if (taps.size() > 9 || taps.empty()) throw std::runtime_error("hwgrad: 1..9 taps");
          a.ntaps = (int)taps.size();
          for (size_t i = 0; i < taps.size(); ++i) { a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; }
          hwgrad(a, splits, S(stream));
        });
  m.def("hwgrad_supported", &hwgrad_supported);
  m.def("hwgrad_s2_supported", &hwgrad_s2_supported);
  m.def("hwgrad_s2_splits", &hwgrad_s2_splits);
  m.def("hwgrad_s2",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, unsigned dy_bytes, unsigned x_bytes, int NB,
           int H, int W, int Cs, int Co, int splits, uintptr_t stream) {
          HWArgs a{};
          a.dY = P<const bf16*>(dY); a.X = P<const bf16*>(X); a.slab = P<float*>(slab);
          a.bias_slab = P<float*>(bias_slab);
          a.dy_bytes = dy_bytes; a.x_bytes = x_bytes;
          a.NB = NB; a.H = H; a.W = W; a.Cs = Cs; a.Co = Co; a.ntaps = 9;
          hwgrad_s2(a, splits, S(stream));
        });
  m.def("hwgrad_f32",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, unsigned dy_bytes, unsigned x_bytes, int NB,
           int H, int W, int Cs, int Co, int splits, uintptr_t stream) {
          HWArgs a{};
          a.dY = P<const bf16*>(dY); a.X = P<const bf16*>(X); a.slab = P<float*>(slab);
          a.bias_slab = P<float*>(bias_slab);
          a.dy_bytes = dy_bytes; a.x_bytes = x_bytes;
          a.NB = NB; a.H = H; a.W = W; a.Cs = Cs; a.Co = Co;
          a.ntaps = 9;
          for (int t = 0; t < 9; ++t) { a.tap_dy[t] = t / 3 - 1; a.tap_dx[t] = t % 3 - 1; }
          hwgrad_f32(a, splits, S(stream));
        });
  m.def("hwgrad_f32_supported", &hwgrad_f32_supported);
  m.def("hwgrad_f32_splits", &hwgrad_f32_splits);
  m.def("split3_bf16", [](uintptr_t in, uintptr_t out, long rows, int C, int pattern, uintptr_t st) {
    split3_bf16(P<const float*>(in), P<bf16*>(out), rows, C, pattern, S(st));
  });
  m.def("hwgrad_splits", &hwgrad_splits);
  m.def("hwgrad_set_version", &hwgrad_set_version);
  m.def("gemm_g2f",
        [](uintptr_t A, uintptr_t B, uintptr_t C, unsigned a_bytes, unsigned b_bytes, int M, int N, int Cs, int H,
           int W, int GH, int GW, int SY, int SX, std::vector<std::array<int, 4>> taps, int ldb, int ldc, int OH,
           int OW, int OSY, int OSX, int ORY, int ORX, uintptr_t bias, uintptr_t residual, uintptr_t stats, int relu,
           uintptr_t zero_ptr, int zero_n, std::array<uintptr_t, 4> bnb, uintptr_t stream) {
          G2Args a{};  // fp32 operands (pointers reinterpreted by the kernel)
          if (bnb[1]) throw std::runtime_error("gemm_g2f: backward-BN epilogue fusion is bf16-only");
          a.A = P<const bf16*>(A); a.B = P<const bf16*>(B); a.C = P<bf16*>(C);
          a.a_bytes = a_bytes; a.b_bytes = b_bytes;
          a.M = M; a.N = N; a.Cs = Cs; a.H = H; a.W = W; a.GH = GH; a.GW = GW; a.SY = SY; a.SX = SX;
          if (taps.size() > 64) throw std::runtime_error("gemm_g2f: more than 64 taps");
          a.ntaps = (int)taps.size();
          for (size_t i = 0; i < taps.size(); ++i) {
            a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; a.tap_srcoff[i] = taps[i][2]; a.tap_b[i] = taps[i][3];
          }
          a.ldb = ldb; a.ldc = ldc; a.OH = OH; a.OW = OW; a.OSY = OSY; a.OSX = OSX; a.ORY = ORY; a.ORX = ORX;
          a.bias = P<const float*>(bias); a.residual = P<const bf16*>(residual); a.stats = P<float*>(stats); a.relu = relu;
          a.zero_ptr = P<float*>(zero_ptr); a.zero_n = zero_n;
          gemm_g2f(a, S(stream));
        });
  m.def("gemm_g2f_stat_rows", &gemm_g2f_stat_rows);
  m.def("gemm_g2_set_splitk", &gemm_g2_set_splitk);  // (DCNN_G2_SPLITK at run time: tests / A/B)
  m.def("gemm_g2_splitk_enabled", &gemm_g2_splitk_enabled);
  m.def("set_f32_mode", &set_f32_mode);
  m.def("get_f32_mode", &get_f32_mode);
  m.def("gemm_t2f",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, int M, int N, int Pn, int ldy, int Cs,
           int H, int W, int GH, int GW, int SY, int SX, std::vector<std::array<int, 2>> taps, int splits,
           uintptr_t stream) {
          T2Args a{};
          a.dY = P<const bf16*>(dY); a.X = P<const bf16*>(X); a.slab = P<float*>(slab); a.bias_slab = P<float*>(bias_slab);
          a.M = M; a.N = N; a.P = Pn; a.ldy = ldy; a.Cs = Cs; a.H = H; a.W = W; a.GH = GH; a.GW = GW; a.SY = SY; a.SX = SX;
          if (taps.size() > 64) throw std::runtime_error("gemm_t2f: more than 64 taps");
          a.ntaps = (int)taps.size();
          for (size_t i = 0; i < taps.size(); ++i) { a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; }
          gemm_t2f(a, splits, S(stream));
        });
  m.def("gemm_t2f_splits", &gemm_t2f_splits);
  m.def("conv_weight_transpose_f32", [](uintptr_t w, uintptr_t wt, int Co, int T_, int Ci, uintptr_t st) {
    conv_weight_transpose_f32(P<const float*>(w), P<float*>(wt), Co, T_, Ci, S(st));
  });
  m.def("gemm_g2", [](uintptr_t A, uintptr_t B, uintptr_t C, unsigned a_bytes, unsigned b_bytes, int M, int N, int Cs,
                      int H, int W, int GH, int GW, int SY, int SX, std::vector<std::array<int, 4>> taps, int ldb,
                      int ldc, int OH, int OW, int OSY, int OSX, int ORY, int ORX, uintptr_t bias, uintptr_t residual,
                      uintptr_t stats, int relu, uintptr_t zero_ptr, int zero_n, std::array<uintptr_t, 4> bnb,
                      uintptr_t stream) {
    bind_gemm_g2(A, B, C, a_bytes, b_bytes, M, N, Cs, H, W, GH, GW, SY, SX, std::move(taps), ldb, ldc, OH, OW, OSY, OSX,
                 ORY, ORX, bias, residual, stats, relu, zero_ptr, zero_n, bnb, stream, {});
  });
  // grouped row classes (strided-dgrad phases in one launch): classes = (first tap, taps, ORY, ORX)
  m.def("gemm_g2_grouped", &bind_gemm_g2);
  m.def("gemm_g2_stat_rows", &gemm_g2_stat_rows);
  for (auto [name, fn] : {std::pair<const char*, int (*)(ConvRouteGeom)>{"conv_fwd_route", &conv_fwd_route},
                          {"conv_dgrad_route", &conv_dgrad_route}, {"conv_wgrad_route", &conv_wgrad_route}})
    m.def(name, [fn](int N, int C, int H, int W, int Co, int KH, int KW, int SH, int SW, int PH, int PW, int OH, int OW,
                     int g1s_mode) { return fn(ConvRouteGeom{N, C, H, W, Co, KH, KW, SH, SW, PH, PW, OH, OW, g1s_mode}); });
  m.attr("ROUTE_GENERIC") = (int)ROUTE_GENERIC;
  m.attr("ROUTE_GEMM_G2") = (int)ROUTE_GEMM_G2;
  m.attr("ROUTE_HALO") = (int)ROUTE_HALO;
  m.attr("ROUTE_G1S") = (int)ROUTE_G1S;
  m.attr("ROUTE_HALO_S2") = (int)ROUTE_HALO_S2;
  // the shared fusion planner (fusion_plan.cpp)
  m.def("plan_sequence_fusions", &plan_sequence_fusions);
  m.def("plan_residual_fusions", &plan_residual_fusions);
  for (auto [name, v] : {std::pair<const char*, int>{"FK_OTHER", FK_OTHER}, {"FK_CONV", FK_CONV}, {"FK_BN", FK_BN},
                         {"FK_RELU", FK_RELU}, {"FK_ACT", FK_ACT}, {"FK_MAXPOOL", FK_MAXPOOL},
                         {"FF_EMIT_BN_STATS", FF_EMIT_BN_STATS}, {"FF_FUSE_RELU", FF_FUSE_RELU},
                         {"FF_PASSTHROUGH", FF_PASSTHROUGH}, {"FF_FUSE_POOL", FF_FUSE_POOL},
                         {"FF_BNB_CONSUMER", FF_BNB_CONSUMER}, {"RF_FUSED_TAIL", RF_FUSED_TAIL},
                         {"RF_DUAL_SHORTCUT", RF_DUAL_SHORTCUT}})
    m.attr(name) = v;
  m.def("g1s_rows", &g1s_rows);
  m.def("g1s_enable", &g1s_enable);
  m.def("g1s_set_waves_per_simd", &g1s_set_waves_per_simd);
  m.def("g1s_gen_rows", &g1s_gen_rows);
  m.def("g1s_gen", [](uintptr_t X, uintptr_t Wt, uintptr_t Y, int NB, int GH, int GW, int N, int Kc, int ldw,
                      std::vector<std::array<int, 3>> taps, int H, int W, int OHo, int OWo, int OS, int ORY, int ORX,
                      uintptr_t residual, uintptr_t stats, uintptr_t zero_ptr, int zero_n, std::array<uintptr_t, 4> bnb,
                      int mode, uintptr_t stream) {
    g1s_gen(P<const bf16*>(X), P<const bf16*>(Wt), P<bf16*>(Y), NB, GH, GW, N, Kc, ldw, taps, H, W, OHo, OWo, OS, ORY,
            ORX, P<const bf16*>(residual), P<float*>(stats), P<float*>(zero_ptr), zero_n,
            BnbArgs{P<const bf16*>(bnb[0]), P<const bf16*>(bnb[1]), P<const float*>(bnb[2]), P<const float*>(bnb[3])},
            mode, S(stream));
  });
  m.def("g1s", [](uintptr_t X, uintptr_t Wt, uintptr_t Y, int M, int N, int K, int H, int W, int OH, int OW, int stride,
                  uintptr_t bias, uintptr_t residual, uintptr_t stats, int relu, uintptr_t zero_ptr, int zero_n,
                  std::array<uintptr_t, 4> bnb, int mode, uintptr_t stream) {
    g1s(P<const bf16*>(X), P<const bf16*>(Wt), P<bf16*>(Y), M, N, K, H, W, OH, OW, stride, P<const float*>(bias),
        P<const bf16*>(residual), P<float*>(stats), relu, P<float*>(zero_ptr), zero_n,
        BnbArgs{P<const bf16*>(bnb[0]), P<const bf16*>(bnb[1]), P<const float*>(bnb[2]), P<const float*>(bnb[3])},
        mode, S(stream));
  });
  m.def("gemm_g2_row_tile", &gemm_g2_row_tile);
  m.def("gemm_t2",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, unsigned a_bytes, unsigned b_bytes, int M,
           int N, int Pn, int ldy, int Cs, int H, int W, int GH, int GW, int SY, int SX,
           std::vector<std::array<int, 2>> taps, int splits, uintptr_t stream) {
          T2Args a{};
          a.dY = P<const bf16*>(dY); a.X = P<const bf16*>(X); a.slab = P<float*>(slab); a.bias_slab = P<float*>(bias_slab);
          a.a_bytes = a_bytes; a.b_bytes = b_bytes; a.M = M; a.N = N; a.P = Pn; a.ldy = ldy; a.Cs = Cs;
          a.H = H; a.W = W; a.GH = GH; a.GW = GW; a.SY = SY; a.SX = SX;
          if (taps.size() > 64) throw std::runtime_error("gemm_t2: more than 64 taps");
          a.ntaps = (int)taps.size();
          for (size_t i = 0; i < taps.size(); ++i) { a.tap_dy[i] = taps[i][0]; a.tap_dx[i] = taps[i][1]; }
          gemm_t2(a, splits, S(stream));
        });
  m.def("gemm_t2_splits", &gemm_t2_splits);
  m.def("gemm_tn",
        [](uintptr_t dY, uintptr_t X, uintptr_t slab, uintptr_t bias_slab, int M, int N, int Pn, int mode, int nb,
           int sh, int sw, int cs, int gh, int gw, int kh, int kw, int strh, int strw, int padh, int padw, int ldx,
           int splits, uintptr_t stream) {
          TnArgs a{P<const bf16*>(dY), P<const bf16*>(X), P<float*>(slab), P<float*>(bias_slab), M, N, Pn, mode, nb, sh,
                   sw, cs, gh, gw, kh, kw, strh, strw, padh, padw, ldx, 0};
          gemm_tn(a, splits, S(stream));
        });
  m.def("gemm_tn_splits", &gemm_tn_splits);
  m.def("splitk_reduce", [](uintptr_t slab, uintptr_t out, long n, int splits, int acc, uintptr_t st) {
    splitk_reduce(P<const float*>(slab), P<float*>(out), n, splits, acc, S(st));
  });
  m.def("splitk_reduce2", [](uintptr_t slab, uintptr_t out, long n, uintptr_t bslab, uintptr_t bout, long nb,
                             int splits, int acc, uintptr_t st) {
    splitk_reduce2(P<const float*>(slab), P<float*>(out), n, P<const float*>(bslab), P<float*>(bout), nb, splits, acc,
                   S(st));
  });

  m.def("bn_partial_rows", &bn_partial_rows);
  m.def("bn_partial", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t yout, uintptr_t dy_out, uintptr_t mean,
                         uintptr_t istd, long R, int C, uintptr_t slab, int mode, uintptr_t zero_sums, uintptr_t st) {
    bn_partial(dt, P<const void*>(x), P<const void*>(dy), P<const void*>(yout), P<void*>(dy_out),
               P<const float*>(mean), P<const float*>(istd), R, C, P<float*>(slab), mode, P<float*>(zero_sums), S(st));
  });
  m.def("bn_stat_parts", &bn_stat_parts);
  m.def("bn_stat_reduce", [](int mode, uintptr_t slab, int rows, int C, uintptr_t out, uintptr_t part, uintptr_t ticket,
                             uintptr_t st) {
    bn_stat_reduce(mode, P<const float*>(slab), rows, C, P<float*>(out), P<float*>(part), P<unsigned*>(ticket), S(st));
  });
  m.def("bn_apply", [](int dt, uintptr_t x, uintptr_t y, long R, int C, uintptr_t sums, int parts, float count,
                       uintptr_t gamma, uintptr_t beta, float eps, uintptr_t residual, int relu, uintptr_t save_mean,
                       uintptr_t save_istd, uintptr_t run_mean, uintptr_t run_var, float momentum, int use_running,
                       uintptr_t st) {
    bn_apply(dt, P<const void*>(x), P<void*>(y), R, C, P<const float*>(sums), parts, count, P<const float*>(gamma),
             P<const float*>(beta), eps, P<const void*>(residual), relu, P<float*>(save_mean), P<float*>(save_istd),
             P<float*>(run_mean), P<float*>(run_var), momentum, use_running, S(st));
  });
  // side = (x, sums, parts, count, gamma, beta, eps, save_mean, save_istd, run_mean, run_var, momentum, use_running)
  using SideT = std::tuple<uintptr_t, uintptr_t, int, float, uintptr_t, uintptr_t, float, uintptr_t, uintptr_t, uintptr_t,
                           uintptr_t, float, int>;
  auto side = [](const SideT& t) {
    BnSide b{};
    b.x = P<const void*>(std::get<0>(t)); b.sums = P<const float*>(std::get<1>(t)); b.parts = std::get<2>(t);
    b.count = std::get<3>(t); b.gamma = P<const float*>(std::get<4>(t)); b.beta = P<const float*>(std::get<5>(t));
    b.eps = std::get<6>(t); b.save_mean = P<float*>(std::get<7>(t)); b.save_istd = P<float*>(std::get<8>(t));
    b.run_mean = P<float*>(std::get<9>(t)); b.run_var = P<float*>(std::get<10>(t)); b.momentum = std::get<11>(t);
    b.use_running = std::get<12>(t);
    return b;
  };
  m.def("bn_apply_dual", [side](SideT a, SideT b, uintptr_t y, long R, int C, int relu, uintptr_t st) {
    return bn_apply_dual(side(a), side(b), P<void*>(y), R, C, relu, S(st));
  });
  m.def("bn_apply_dual_supported", &bn_apply_dual_supported);
  // bside = (x, dx, mean, istd, gamma, sums, parts, count, dgamma, dbeta)
  using BSideT = std::tuple<uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, float, uintptr_t,
                            uintptr_t>;
  auto bside = [](const BSideT& t) {
    BnBwdSide b{};
    b.x = P<const void*>(std::get<0>(t)); b.dx = P<void*>(std::get<1>(t)); b.mean = P<const float*>(std::get<2>(t));
    b.istd = P<const float*>(std::get<3>(t)); b.gamma = P<const float*>(std::get<4>(t));
    b.sums = P<const float*>(std::get<5>(t)); b.parts = std::get<6>(t); b.count = std::get<7>(t);
    b.dgamma = P<float*>(std::get<8>(t)); b.dbeta = P<float*>(std::get<9>(t));
    return b;
  };
  m.def("bn_bwd_apply_dual", [bside](uintptr_t dy, BSideT a, BSideT b, long R, int C, uintptr_t st) {
    return bn_bwd_apply_dual(P<const void*>(dy), bside(a), bside(b), R, C, S(st));
  });
  m.def("bn_stat_reduce2", [](int mode, uintptr_t slab, int rows, uintptr_t out, uintptr_t part, uintptr_t slab2, int rows2,
                              uintptr_t out2, uintptr_t part2, int C, uintptr_t st) {
    bn_stat_reduce2(mode, P<const float*>(slab), rows, P<float*>(out), P<float*>(part), P<const float*>(slab2), rows2,
                    P<float*>(out2), P<float*>(part2), C, S(st));
  });
  m.def("bn_bwd_apply", [](int dt, uintptr_t dy, uintptr_t yout, uintptr_t x, uintptr_t dx, long R, int C,
                           uintptr_t mean, uintptr_t istd, uintptr_t gamma, uintptr_t sums, int parts, float count,
                           uintptr_t dgamma, uintptr_t dbeta, int eval_mode, uintptr_t st) {
    bn_bwd_apply(dt, P<const void*>(dy), P<const void*>(yout), P<const void*>(x), P<void*>(dx), R, C,
                 P<const float*>(mean), P<const float*>(istd), P<const float*>(gamma), P<const float*>(sums), parts,
                 count,
                 P<float*>(dgamma), P<float*>(dbeta), eval_mode, S(st));
  });
  m.def("gn_fwd", [](int dt, uintptr_t x, uintptr_t y, int N, int HW, int C, int G, uintptr_t gamma, uintptr_t beta,
                     float eps, uintptr_t sm, uintptr_t si, uintptr_t st) {
    gn_fwd(dt, P<const void*>(x), P<void*>(y), N, HW, C, G, P<const float*>(gamma), P<const float*>(beta), eps,
           P<float*>(sm), P<float*>(si), S(st));
  });
  m.def("gn_bwd", [](int dt, uintptr_t dy, uintptr_t x, uintptr_t dx, int N, int HW, int C, int G, uintptr_t gamma,
                     uintptr_t mean, uintptr_t istd, uintptr_t dg, uintptr_t db, uintptr_t aff, uintptr_t st) {
    gn_bwd(dt, P<const void*>(dy), P<const void*>(x), P<void*>(dx), N, HW, C, G, P<const float*>(gamma),
           P<const float*>(mean), P<const float*>(istd), P<float*>(dg), P<float*>(db), P<float*>(aff), S(st));
  });

  auto geom = [](int N, int H, int W, int C, int OH, int OW, int ph, int pw, int sh, int sw, int padh, int padw) {
    return PoolGeom{N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw};
  };
  m.def("maxpool_fwd", [geom](int dt, uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int OH,
                              int OW, int ph, int pw, int sh, int sw, int padh, int padw, uintptr_t st) {
    maxpool_fwd(dt, P<const void*>(x), P<void*>(y), P<uint8_t*>(idx), geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw),
                S(st));
  });
  m.def("maxpool_bwd", [geom](int dt, uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C, int OH,
                              int OW, int ph, int pw, int sh, int sw, int padh, int padw, uintptr_t st) {
    maxpool_bwd(dt, P<const void*>(dy), P<const uint8_t*>(idx), P<void*>(dx),
                geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw), S(st));
  });
  m.def("maxpool_bwd_bnb_supported", [geom](int N, int H, int W, int C, int OH, int OW, int ph, int pw, int sh, int sw,
                                            int padh, int padw) {
    return maxpool_bwd_bnb_supported(geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw));
  });
  m.def("bn_relu_maxpool_supported", [geom](int N, int H, int W, int C, int OH, int OW, int ph, int pw, int sh, int sw,
                                            int padh, int padw) {
    return bn_relu_maxpool_supported(geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw));
  });
  m.def("bn_relu_maxpool", [geom](uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int OH, int OW,
                                  int ph, int pw, int sh, int sw, int padh, int padw, uintptr_t sums, int parts,
                                  float count,
                                  uintptr_t gamma, uintptr_t beta, float eps, uintptr_t save_mean, uintptr_t save_istd,
                                  uintptr_t run_mean, uintptr_t run_var, float momentum, uintptr_t st) {
    bn_relu_maxpool(P<const bf16*>(x), P<bf16*>(y), P<uint8_t*>(idx), geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw),
                    P<const float*>(sums), parts, count, P<const float*>(gamma), P<const float*>(beta), eps,
                    P<float*>(save_mean), P<float*>(save_istd), P<float*>(run_mean), P<float*>(run_var), momentum,
                    S(st));
  });
  m.def("maxpool_bwd_bnb_rows", [geom](int N, int H, int W, int C, int OH, int OW, int ph, int pw, int sh, int sw,
                                       int padh, int padw) {
    return maxpool_bwd_bnb_rows(geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw));
  });
  m.def("maxpool_bwd_bnb", [geom](uintptr_t dy, uintptr_t idx, uintptr_t ypool, uintptr_t x, uintptr_t mean,
                                  uintptr_t istd, uintptr_t dx, int N, int H, int W, int C, int OH, int OW, int ph,
                                  int pw, int sh, int sw, int padh, int padw, uintptr_t slab, uintptr_t zero_sums,
                                  uintptr_t st) {
    maxpool_bwd_bnb(P<const bf16*>(dy), P<const uint8_t*>(idx), P<const bf16*>(ypool), P<const bf16*>(x),
                    P<const float*>(mean), P<const float*>(istd), P<bf16*>(dx),
                    geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw), P<float*>(slab), P<float*>(zero_sums), S(st));
  });
  m.def("avgpool_fwd", [geom](int dt, uintptr_t x, uintptr_t y, int N, int H, int W, int C, int OH, int OW, int ph,
                              int pw, int sh, int sw, int padh, int padw, uintptr_t st) {
    avgpool_fwd(dt, P<const void*>(x), P<void*>(y), geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw), S(st));
  });
  m.def("avgpool_bwd", [geom](int dt, uintptr_t dy, uintptr_t dx, int N, int H, int W, int C, int OH, int OW, int ph,
                              int pw, int sh, int sw, int padh, int padw, uintptr_t st) {
    avgpool_bwd(dt, P<const void*>(dy), P<void*>(dx), geom(N, H, W, C, OH, OW, ph, pw, sh, sw, padh, padw), S(st));
  });
  m.def("act_fwd", [](int dt, uintptr_t x, uintptr_t y, long n, int type, float a, uintptr_t st) {
    act_fwd(dt, P<const void*>(x), P<void*>(y), n, type, a, S(st));
  });
  m.def("act_bwd", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t dx, long n, int type, float a, uintptr_t st) {
    act_bwd(dt, P<const void*>(x), P<const void*>(dy), P<void*>(dx), n, type, a, S(st));
  });
  m.def("softmax_rows", [](int dt, uintptr_t x, uintptr_t y, long rows, int C, uintptr_t st) {
    softmax_rows(dt, P<const void*>(x), P<void*>(y), rows, C, S(st));
  });
  m.def("softmax_rows_bwd", [](int dt, uintptr_t y, uintptr_t dy, uintptr_t dx, long rows, int C, uintptr_t st) {
    softmax_rows_bwd(dt, P<const void*>(y), P<const void*>(dy), P<void*>(dx), rows, C, S(st));
  });
  m.def("dropout", [](int dt, uintptr_t x, uintptr_t y, long n, float p, uint64_t seed, uintptr_t ctr, uintptr_t st) {
    dropout(dt, P<const void*>(x), P<void*>(y), n, p, seed, P<const uint64_t*>(ctr), S(st));
  });
  m.def("counter_bump", [](uintptr_t ctr, uintptr_t slot, uintptr_t st) {
    counter_bump(P<uint64_t*>(ctr), P<uint64_t*>(slot), S(st));
  });
  m.def("nchw_to_nhwc", [](int dt, uintptr_t x, uintptr_t y, int N, int C, int HW, uintptr_t st) {
    nchw_to_nhwc(dt, P<const float*>(x), P<void*>(y), N, C, HW, S(st));
  });
  m.def("nchw_to_nhwc_pad", [](int dt, uintptr_t x, uintptr_t y, int N, int C, int Cp, int HW, uintptr_t st) {
    nchw_to_nhwc_pad(dt, P<const float*>(x), P<void*>(y), N, C, Cp, HW, S(st));
  });
  m.def("conv_weight_transpose", [](int dt, uintptr_t w, uintptr_t wt, int Co, int T_, int Ci, uintptr_t st) {
    conv_weight_transpose(dt, P<const void*>(w), P<bf16*>(wt), Co, T_, Ci, S(st));
  });
  m.def("multi_splitk_reduce", [](std::vector<std::array<int64_t, 4>> ents, uintptr_t st) {
    // entries: (slab ptr, out ptr, n, splits); launched in batches of kMaxRed
    for (size_t b = 0; b < ents.size(); b += kMaxRed) {
      MultiRed t{};
      t.count = (int)std::min(ents.size() - b, (size_t)kMaxRed);
      for (int k = 0; k < t.count; ++k) {
        const auto& e = ents[b + k];
        t.e[k].slab = P<const float*>((uintptr_t)e[0]); t.e[k].out = P<float*>((uintptr_t)e[1]);
        t.e[k].n = e[2]; t.e[k].splits = (int)e[3];
      }
      multi_splitk_reduce(t, S(st));
    }
  });
  m.def("multi_red_max", []() { return kMaxRed; });
  m.def("stem_supported", &stem_supported);
  m.def("stem_tiles", &stem_tiles_host);
  m.def("stem_wgrad_blocks", &stem_wgrad_blocks);
  m.def("stem_fwd", [](uintptr_t x, uintptr_t w, int w_bf16, std::array<long, 4> ws, uintptr_t bias, uintptr_t y,
                       uintptr_t slab, uintptr_t zero_ptr, int zero_n, int N, int Ci, int H, int W, int Co,
                       uintptr_t st) {
    StemArgs a{};
    a.x = P<const float*>(x); a.w = P<const void*>(w); a.w_bf16 = w_bf16;
    for (int i = 0; i < 4; ++i) a.ws[i] = ws[i];
    a.bias = P<const float*>(bias); a.y = P<bf16*>(y); a.slab = P<float*>(slab);
    a.zero_ptr = P<float*>(zero_ptr); a.zero_n = zero_n;
    a.N = N; a.Ci = Ci; a.H = H; a.W = W; a.Co = Co;
    stem_fwd(a, S(st));
  });
  m.def("stem_wgrad", [](uintptr_t x, uintptr_t dy, uintptr_t slab, uintptr_t bias_slab, std::array<long, 4> gs,
                         int N, int Ci, int H, int W, int Co, int blocks, uintptr_t st) {
    StemArgs a{};
    a.x = P<const float*>(x); a.dy = P<const bf16*>(dy); a.slab = P<float*>(slab);
    a.bias_slab = P<float*>(bias_slab);
    for (int i = 0; i < 4; ++i) a.gs[i] = gs[i];
    a.n_slab = (long)Co * Ci * 9;
    a.N = N; a.Ci = Ci; a.H = H; a.W = W; a.Co = Co;
    stem_wgrad(a, blocks, S(st));
  });
  m.def("multi_weight_transpose", [](uintptr_t table, int n, long max_tiles, uintptr_t st, int f32) {
    multi_weight_transpose(P<const int64_t*>(table), n, max_tiles, S(st), f32);
  });
  m.def("cast_f32_bf16",[](uintptr_t x, uintptr_t y, long n, uintptr_t st) {
    cast_f32_bf16(P<const float*>(x), P<bf16*>(y), n, S(st));
  });
  m.def("im2col_nhwc", [](int dt, uintptr_t x, uintptr_t col, int N, int H, int W, int C, int OH, int OW, int KH, int KW,
                          int SH, int SW, int PH, int PW, uintptr_t st) {
    im2col_nhwc(dt, P<const void*>(x), P<void*>(col), ConvGeom{N, H, W, C, OH, OW, KH, KW, SH, SW, PH, PW}, S(st));
  });
  m.def("col2im_nhwc", [](int dt, uintptr_t col, uintptr_t x, uintptr_t residual, int N, int H, int W, int C, int OH,
                          int OW, int KH, int KW, int SH, int SW, int PH, int PW, int chan_major, uintptr_t st) {
    col2im_nhwc(dt, P<const void*>(col), P<void*>(x), P<const void*>(residual),
                ConvGeom{N, H, W, C, OH, OW, KH, KW, SH, SW, PH, PW}, chan_major, S(st));
  });
  m.def("im2col", [](uintptr_t x, uintptr_t col, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH,
                     int PW, int OH, int OW, uintptr_t st) {
    im2col(P<const float*>(x), P<float*>(col), N, C, H, W, KH, KW, SH, SW, PH, PW, OH, OW, S(st));
  });
  m.def("col2im", [](uintptr_t col, uintptr_t x, int N, int C, int H, int W, int KH, int KW, int SH, int SW, int PH,
                     int PW, int OH, int OW, uintptr_t st) {
    col2im(P<const float*>(col), P<float*>(x), N, C, H, W, KH, KW, SH, SW, PH, PW, OH, OW, S(st));
  });
  m.def("loss_workspace_floats", &loss_workspace_floats);
  m.def("loss_fused", [](int dt, uintptr_t pred, uintptr_t target, uintptr_t labels, uintptr_t grad, uintptr_t loss,
                         uintptr_t correct, int N, int C, int type, float param, float gscale, uintptr_t ws,
                         uintptr_t ticket, uintptr_t st) {
    loss_fused(dt, P<const void*>(pred), P<const float*>(target), P<const int64_t*>(labels), P<void*>(grad),
               P<float*>(loss), P<int*>(correct), N, C, type, param, gscale, P<float*>(ws), P<unsigned*>(ticket),
               S(st));
  });
  m.def("adam_step", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t shadow, long n, float lr,
                        float b1, float b2, float eps, float bc1, float bc2, float wd, int dec, uintptr_t hyper,
                        uintptr_t st) {
    adam_step(P<float*>(p), P<const float*>(g), P<float*>(mm), P<float*>(v), P<bf16*>(shadow), n, lr, b1, b2, eps, bc1,
              bc2, wd, dec, P<const float*>(hyper), S(st));
  });
  m.def("adam_scalars", [](uintptr_t hyper, float b1, float b2, uintptr_t st) {
    adam_scalars(P<float*>(hyper), b1, b2, S(st));
  });
  m.def("sgd_step", [](uintptr_t p, uintptr_t g, uintptr_t vel, uintptr_t shadow, long n, float lr, float mom,
                       uintptr_t hyper, uintptr_t st) {
    sgd_step(P<float*>(p), P<const float*>(g), P<float*>(vel), P<bf16*>(shadow), n, lr, mom, P<const float*>(hyper),
             S(st));
  });
  m.def("zero_bytes", [](uintptr_t p, long nbytes, uintptr_t st) { zero_bytes(P<void*>(p), nbytes, S(st)); });
  m.def("grad_pack_bf16", [](uintptr_t g, uintptr_t out, long n, float scale, uintptr_t st) {
    grad_pack_bf16(P<const float*>(g), P<bf16*>(out), n, scale, S(st));
  });
  m.def("grad_sum_chunks_bf16", [](uintptr_t src, int w, long ld, long n, uintptr_t dst, uintptr_t st) {
    grad_sum_chunks_bf16(P<const bf16*>(src), w, ld, n, P<bf16*>(dst), S(st));
  });
  m.def("grad_unpack_bf16", [](uintptr_t in, uintptr_t g, long n, uintptr_t st) {
    grad_unpack_bf16(P<const bf16*>(in), P<float*>(g), n, S(st));
  });
  m.def("augment_batch_supported", &augment_batch_supported);
  // ops: (kind, probability, params[<= 6]) in chain order
  m.def("augment_batch", [](uintptr_t src, int src_u8, uintptr_t idx, uintptr_t labels, uintptr_t labels_out,
                            uintptr_t out, int B, int C, int H, int W, unsigned long long seed,
                            const std::vector<std::tuple<int, float, std::vector<float>>>& ops, uintptr_t st) {
    AugBatchArgs a{};
    a.src = P<const void*>(src); a.src_u8 = src_u8; a.idx = P<const int64_t*>(idx);
    a.labels = P<const int64_t*>(labels); a.labels_out = P<int64_t*>(labels_out); a.out = P<float*>(out);
    a.B = B; a.C = C; a.H = H; a.W = W; a.seed = seed;
    if (ops.size() > (size_t)kAugMaxOps) throw std::runtime_error("augment_batch: at most 12 ops");
    a.nops = (int)ops.size();
    for (size_t k = 0; k < ops.size(); ++k) {
      a.ops[k].kind = std::get<0>(ops[k]);
      a.ops[k].p = std::get<1>(ops[k]);
      const auto& v = std::get<2>(ops[k]);
      if (v.size() > 6) throw std::runtime_error("augment_batch: at most 6 op parameters");
      for (size_t j = 0; j < v.size(); ++j) a.ops[k].a[j] = v[j];
    }
    augment_batch(a, S(st));
  });
  m.attr("AUG_KINDS") = py::make_tuple("horizontal_flip", "vertical_flip", "rotation", "brightness", "contrast",
                                       "gaussian_noise", "random_crop", "cutout", "normalize");
}
