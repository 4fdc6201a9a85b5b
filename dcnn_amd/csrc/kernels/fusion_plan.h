// The shared fusion planner (fusion_plan.cpp): the cross-layer fusions of a layer sequence on the
// GPU path, one rule set for both front ends (the Python layers and the C++ host API). Plain C++
// (no HIP types), so host-only translation units include it too.
#pragma once
#include <vector>

namespace dcnn {

// layer kinds in order -> per-layer FF_* flags
enum FuseKind : int { FK_OTHER = 0, FK_CONV = 1, FK_BN = 2, FK_RELU = 3, FK_ACT = 4, FK_MAXPOOL = 5 };
enum FuseFlag : int {
  FF_EMIT_BN_STATS = 1,  // conv: its epilogue emits the statistics rows of the BatchNorm after it
  FF_FUSE_RELU = 2,      // BatchNorm: its apply pass applies the ReLU after it
  FF_PASSTHROUGH = 4,    // ReLU: already applied by the BatchNorm before it
  FF_FUSE_POOL = 8,      // BatchNorm: its training apply also runs the max-pool two layers on
  FF_BNB_CONSUMER = 16,  // conv: its data gradient carries the backward of the BatchNorm [+ ReLU] before it
};
std::vector<int> plan_sequence_fusions(const std::vector<int>& kinds);
// residual block (main path kinds, shortcut kinds, block activation relu / linear / none):
// RF_FUSED_TAIL = the main path's closing BatchNorm applies the shortcut sum and the activation;
// RF_DUAL_SHORTCUT = the shortcut's closing BatchNorm shares that pass
enum ResidualFlag : int { RF_FUSED_TAIL = 1, RF_DUAL_SHORTCUT = 2 };
int plan_residual_fusions(const std::vector<int>& main_kinds, const std::vector<int>& short_kinds, bool act_ok);

}  // namespace dcnn
