// The shared fusion planner (api.h): which cross-layer fusions a layer sequence gets on the GPU
// path, decided in one place for both front ends — the Python layers (nn/layers/residual.py
// plan_fusion, ResidualBlock._plan) and the C++ host API (csrc/host/nn.cpp fuse_bn_relu,
// ResidualBlock::fused_tail / dual_shortcut). Like the conv routing table (conv_route.cpp) it
// sees only what both front ends can describe: the kinds of the layers in order.
//
// Reference parity: the reference runs every layer as its own kernels (no cross-layer fusion,
// src/nn/layers_impl/cuda/batchnorm_ops.cu:297-324 is a standalone pass); SURVEY §7.1 lists
// these fusions as the MI355X design.
#include "fusion_plan.h"

namespace dcnn {

std::vector<int> plan_sequence_fusions(const std::vector<int>& kinds) {
  const size_t n = kinds.size();
  std::vector<int> f(n, 0);
  auto is = [&](size_t i, int k) { return i < n && kinds[i] == k; };
  for (size_t i = 0; i + 1 < n; ++i) {
    // conv -> BatchNorm: the conv's epilogue emits the BatchNorm's statistics rows
    if (is(i, FK_CONV) && is(i + 1, FK_BN)) f[i] |= FF_EMIT_BN_STATS;
    // BatchNorm -> ReLU: one apply pass, the ReLU layer passes through
    if (is(i, FK_BN) && is(i + 1, FK_RELU)) {
      f[i] |= FF_FUSE_RELU;
      f[i + 1] |= FF_PASSTHROUGH;
    }
  }
  for (size_t i = 0; i + 2 < n; ++i)  // BatchNorm -> ReLU -> max-pool: the pool inside the apply
    if (is(i, FK_BN) && is(i + 1, FK_RELU) && is(i + 2, FK_MAXPOOL)) f[i] |= FF_FUSE_POOL;
  // BatchNorm [-> ReLU] -> conv: the conv's data gradient carries the BatchNorm backward (ReLU
  // mask + statistics rows) in its epilogue
  for (size_t j = 1; j < n; ++j) {
    if (!is(j, FK_CONV)) continue;
    if (is(j - 1, FK_BN) || (j >= 2 && is(j - 1, FK_RELU) && is(j - 2, FK_BN))) f[j] |= FF_BNB_CONSUMER;
  }
  return f;
}

int plan_residual_fusions(const std::vector<int>& main_kinds, const std::vector<int>& short_kinds, bool act_ok) {
  // the main path's closing BatchNorm applies the shortcut sum and the block activation
  const bool tail = act_ok && main_kinds.size() >= 2 && main_kinds.back() == FK_BN;
  if (!tail) return 0;
  // a projection shortcut's closing BatchNorm is applied in that same pass
  const bool dual = !short_kinds.empty() && short_kinds.back() == FK_BN;
  return RF_FUSED_TAIL | (dual ? RF_DUAL_SHORTCUT : 0);
}

}  // namespace dcnn
