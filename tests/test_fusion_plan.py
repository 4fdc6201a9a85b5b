"""The shared fusion planner (csrc/kernels/fusion_plan.cpp): one rule set for the Python layers
(nn/layers/residual.py plan_fusion, ResidualBlock._plan) and the C++ host API (nn.cpp
fuse_bn_relu, ResidualBlock::fused_tail / dual_shortcut). CPU: the planner is plain C++."""
import pytest

from dcnn_amd.ops._ext import kernels


@pytest.fixture(scope="module")
def K():
    return kernels()


def test_sequence_rules(K):
    C, B, R, A, P, O = K.FK_CONV, K.FK_BN, K.FK_RELU, K.FK_ACT, K.FK_MAXPOOL, K.FK_OTHER
    # stem conv -> BN -> ReLU -> max-pool, then conv -> BN -> ReLU -> conv, a tanh, a BN -> conv
    kinds = [C, B, R, P, C, B, R, C, A, B, C, O]
    f = K.plan_sequence_fusions(kinds)
    assert len(f) == len(kinds)
    assert f[0] == K.FF_EMIT_BN_STATS
    assert f[1] == K.FF_FUSE_RELU | K.FF_FUSE_POOL
    assert f[2] == K.FF_PASSTHROUGH and f[3] == 0
    assert f[4] == K.FF_EMIT_BN_STATS  # (after a max-pool: no backward-BatchNorm producer)
    assert f[5] == K.FF_FUSE_RELU and f[6] == K.FF_PASSTHROUGH
    assert f[7] == K.FF_BNB_CONSUMER  # BN -> ReLU -> conv
    assert f[8] == 0 and f[9] == 0  # a non-ReLU activation breaks both chains
    assert f[10] == K.FF_BNB_CONSUMER  # BN -> conv
    assert f[11] == 0
    assert K.plan_sequence_fusions([]) == [] and K.plan_sequence_fusions([B]) == [0]


def test_residual_rules(K):
    C, B, R = K.FK_CONV, K.FK_BN, K.FK_RELU
    basic, proj = [C, B, R, C, B], [C, B]
    assert K.plan_residual_fusions(basic, proj, True) == K.RF_FUSED_TAIL | K.RF_DUAL_SHORTCUT
    assert K.plan_residual_fusions(basic, [], True) == K.RF_FUSED_TAIL
    assert K.plan_residual_fusions(basic, proj, False) == 0  # an activation the tail pass cannot apply
    assert K.plan_residual_fusions([C, B, R, C], proj, True) == 0  # main path does not end in a BatchNorm
    assert K.plan_residual_fusions([B], [], True) == 0  # (a one-layer main path is not fused)


def test_python_layers_follow_the_planner(K):
    """plan_fusion / ResidualBlock._plan on a GPU-flagged ResNet-18 block set the attributes the
    planner's flags name (no GPU needed: only the planning runs)."""
    from dcnn_amd.nn.layers.conv import Conv2D
    from dcnn_amd.nn.layers.misc import Activation, MaxPool2D
    from dcnn_amd.nn.layers.norm import BatchNorm
    from dcnn_amd.nn.layers.residual import plan_fusion
    seq = [Conv2D(3, 8, 3, 3, 1, 1, 1, 1), BatchNorm(8), Activation("relu"), MaxPool2D(2, 2, 2, 2)]
    plan_fusion(seq, on_gpu=True)
    assert seq[0].emit_bn_stats and seq[1].fuse_relu and seq[2].passthrough and seq[1].fuse_pool is seq[3]
    plan_fusion(seq, on_gpu=False)
    assert not seq[0].emit_bn_stats and not seq[1].fuse_relu and not seq[2].passthrough and seq[1].fuse_pool is None
