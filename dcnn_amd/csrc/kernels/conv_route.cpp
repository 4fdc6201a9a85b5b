// The conv routing table, shared by the Python front end (ops/hip.py) and the C++ host API's GPU
// backend (csrc/host/ops_gpu.hip): which kernel family runs a bf16 convolution. One place decides,
// so both front ends run the same kernels for the same layer.
//
// Reference parity: the reference picks im2col + cuBLAS or cuDNN per layer
// (src/nn/layers_impl/cuda/conv2d_ops.cu:18-128, cudnn_conv2d_ops.cu:187-244).
#include "api.h"

namespace dcnn {

namespace {
bool same_reach1(const ConvRouteGeom& g) {
  // stride 1, output size = input size, every tap within one pixel
  return g.SH == 1 && g.SW == 1 && g.OH == g.H && g.OW == g.W && g.KH <= 3 && g.KW <= 3 && g.KH == 2 * g.PH + 1 &&
         g.KW == 2 * g.PW + 1;
}
// 1x1 convs with K >= 1024 input channels (not on the streaming kernel) whose gathered-GEMM grid
// would be < 256 tiles: the halo kernel splits their K over the channel chunks
// (ResNet-50 b32: 7.87k -> 7.92k img/s)
bool halo_1x1(int M, int K, int N) { return K >= 1024 && (long)(M / 64) * (N / 64) < 256; }
}  // namespace

// the halo_1x1 shapes on the gathered GEMM's split-K path instead (gemm2.hip g2_ksplit: K slices
// over ~512 workgroups + one epilogue launch; ResNet-50 b32 K >= 1024 1x1 convs)
static bool splitk_1x1(int M, int K, int N) {
  return gemm_g2_splitk_enabled() && halo_1x1(M, K, N) && K % 8 == 0 && N % 8 == 0;
}

int conv_fwd_route(ConvRouteGeom g) {
  const int M = g.N * g.OH * g.OW, T = g.KH * g.KW;
  if (g.KH == 1 && g.KW == 1 && g.PH == 0 && g.PW == 0 && g.SH == g.SW && g.g1s_mode >= 0 &&
      g1s_rows(M, g.Co, g.C, g.g1s_mode) > 0)
    return ROUTE_G1S;
  if (T == 1 && g.SH == 1 && g.SW == 1 && g.PH == 0 && g.PW == 0 && splitk_1x1(M, g.C, g.Co)) return ROUTE_GEMM_G2;
  if (same_reach1(g) && (T > 1 || halo_1x1(M, g.C, g.Co)) && hconv_supported(g.N, g.H, g.W, g.C, g.Co, T))
    return ROUTE_HALO;
  if (g.C % 8 == 0 && g.Co % 8 == 0 && T <= 64) return ROUTE_GEMM_G2;
  return ROUTE_GENERIC;
}

int conv_dgrad_route(ConvRouteGeom g) {
  const int M = g.N * g.H * g.W, T = g.KH * g.KW;
  if (T == 1 && g.SH == 1 && g.SW == 1 && g.PH == 0 && g.PW == 0 && splitk_1x1(M, g.Co, g.C)) return ROUTE_GEMM_G2;
  // the data gradient of a 'same' stride-1 conv is a 'same' conv of dY with the flipped taps
  if (same_reach1(g) && (T > 1 || halo_1x1(M, g.Co, g.C)) && hconv_supported(g.N, g.H, g.W, g.Co, g.C, T))
    return ROUTE_HALO;
  if (g.KH == 1 && g.KW == 1 && g.PH == 0 && g.PW == 0 && g.SH == 1 && g.SW == 1 && g.g1s_mode >= 0 &&
      g1s_rows(M, g.C, g.Co, g.g1s_mode) > 0)
    return ROUTE_G1S;
  if (g.C % 8 == 0 && g.Co % 8 == 0 && T <= 64) return ROUTE_GEMM_G2;  // (stride phases grouped)
  return ROUTE_GENERIC;
}

int conv_wgrad_route(ConvRouteGeom g) {
  if (same_reach1(g) && g.KH == 3 && g.KW == 3 && hwgrad_supported(g.N, g.H, g.W, g.C, g.Co, 9)) return ROUTE_HALO;
  // 3x3 stride-2 pad-1 downsampling convs: the stride-2 halo kernel (hwgrad_s2; ResNet-18 b256
  // 85.0k -> 86.4k img/s over gemm_t2, profiles/experiment_hwgrad_s2_r5.md)
  if (g.KH == 3 && g.KW == 3 && g.SH == 2 && g.SW == 2 && g.PH == 1 && g.PW == 1 && g.H == 2 * g.OH &&
      g.W == 2 * g.OW && hwgrad_s2_supported(g.N, g.OH, g.OW, g.C, g.Co))
    return ROUTE_HALO_S2;
  if (g.C % 8 == 0 && g.Co % 8 == 0 && g.KH * g.KW <= 64) return ROUTE_GEMM_G2;  // gemm_t2
  return ROUTE_GENERIC;
}

}  // namespace dcnn
