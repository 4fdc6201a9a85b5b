"""Layer-by-layer suite modelled on the reference's unit tests:

* analytic / autograd references on the CPU device for every layer type and the shapes the
  reference exercises (`unit_tests/conv2d_layer_test.cpp:660-990` ResNet shapes: 1x1 up/down,
  strided, 7x7 stem, asymmetric stride, small maps; `dense_layer_test.cpp`,
  `batchnorm_layer_test.cpp`, `maxpool/avgpool`, `residual_block`, `sequential_residual_block_test.cpp`);
* FLOP / output-shape bookkeeping, gradient accumulation across micro-batches, buffer-reuse
  consistency (`layer_buffer_reuse_test.cpp`), device manager (`device_manager_test.cpp`);
* CPU-vs-GPU "device agnosticity" (`layer_device_agnosticity_test.cpp:60-654`): the same layer
  built on both devices with identical weights, fp32 (tight) and bf16 (loose) GPU compute.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from dcnn_amd.nn import (Activation, AvgPool2D, BatchNorm, Conv2D, Dense, Dropout, Flatten, GroupNorm, LayerBuilder,
                         MaxPool2D, ResidualBlock, Sequential, SequentialBuilder)


def _close(a, b, tol):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return (a - b).norm().item() <= tol * max(b.norm().item(), 1e-6)


# --------------------------------------------------------------------------------- Conv2D
CONV_SHAPES = [
    # N, C, H, W, Co, kh, kw, sh, sw, ph, pw, bias
    (1, 1, 5, 5, 1, 3, 3, 1, 1, 0, 0, True),        # basic 3x3 valid
    (2, 3, 8, 8, 4, 3, 3, 1, 1, 1, 1, True),        # same padding
    (2, 4, 9, 9, 6, 3, 3, 2, 2, 1, 1, True),        # strided odd size
    (1, 8, 6, 6, 16, 1, 1, 1, 1, 0, 0, True),       # 1x1 channel up
    (2, 16, 8, 8, 8, 1, 1, 1, 1, 0, 0, False),      # 1x1 channel down, no bias
    (2, 16, 8, 8, 32, 1, 1, 2, 2, 0, 0, False),     # 1x1 stride-2 projection
    (1, 3, 14, 14, 8, 7, 7, 2, 2, 3, 3, True),      # 7x7 ImageNet stem
    (2, 2, 7, 9, 3, 3, 3, 1, 1, 1, 1, True),        # non-square input
    (1, 4, 10, 12, 5, 3, 3, 2, 1, 1, 1, True),      # asymmetric stride
    (1, 4, 9, 9, 5, 3, 5, 1, 1, 1, 2, True),        # asymmetric kernel / padding
    (2, 32, 4, 4, 32, 3, 3, 1, 1, 1, 1, True),      # small feature map (layer-4 like)
    (1, 64, 2, 2, 16, 3, 3, 1, 1, 1, 1, False),     # 2x2 map, pad dominates
    (3, 5, 6, 6, 7, 2, 2, 2, 2, 0, 0, True),        # 2x2 stride-2 (patchify)
    (1, 2, 5, 5, 3, 5, 5, 1, 1, 0, 0, True),        # kernel == image (1x1 output)
    (2, 6, 8, 8, 6, 3, 3, 3, 3, 0, 0, True),        # stride 3
]


@pytest.mark.parametrize("cfg", CONV_SHAPES)
def test_conv2d_vs_autograd(cfg):
    N, C, H, W, Co, kh, kw, sh, sw, ph, pw, bias = cfg
    conv = Conv2D(C, Co, kh, kw, sh, sw, ph, pw, bias, "c")
    conv.set_seed(11)
    conv.initialize()
    x = torch.randn(N, C, H, W)
    y = conv.forward(x)
    assert list(y.shape) == conv.compute_output_shape(list(x.shape))
    xr = x.clone().requires_grad_(True)
    wr = conv.weights.detach().clone().requires_grad_(True)
    br = conv.bias.detach().view(-1).clone().requires_grad_(True) if bias else None
    ref = F.conv2d(xr, wr, br, (sh, sw), (ph, pw))
    assert torch.allclose(y, ref, atol=1e-4)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    dx = conv.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    assert torch.allclose(conv.gradients()[0], wr.grad, atol=1e-4)
    if bias:
        assert torch.allclose(conv.gradients()[1].view(-1), br.grad, atol=1e-4)


@pytest.mark.parametrize("cfg", CONV_SHAPES[:6])
def test_conv2d_flops_and_config(cfg):
    N, C, H, W, Co, kh, kw, sh, sw, ph, pw, bias = cfg
    conv = Conv2D(C, Co, kh, kw, sh, sw, ph, pw, bias, "c")
    OH, OW = (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1
    macs = N * OH * OW * Co * C * kh * kw
    assert conv.forward_flops([N, C, H, W]) == 2 * macs + (N * OH * OW * Co if bias else 0)
    assert conv.backward_flops([N, C, H, W]) == 4 * macs + (N * OH * OW * Co if bias else 0)
    cfgd = conv.get_config()
    again = Conv2D.from_config(cfgd)
    assert again.get_config() == cfgd


def test_conv2d_microbatch_caches_and_accumulation():
    """Several in-flight micro-batches per layer (pipeline semantics); weight gradients accumulate
    until cleared (reference beta = 1 GEMMs)."""
    conv = Conv2D(3, 4, 3, 3, 1, 1, 1, 1, True, "c")
    conv.set_seed(2)
    conv.initialize()
    xs = [torch.randn(2, 3, 6, 6) for _ in range(3)]
    ys = [conv.forward(x, mb) for mb, x in enumerate(xs)]
    gw = torch.zeros_like(conv.weights)
    for mb in (2, 0, 1):
        dy = torch.ones_like(ys[mb])
        conv.backward(dy, mb)
        gw += torch.nn.grad.conv2d_weight(xs[mb], conv.weights.shape, dy, 1, 1)
    assert torch.allclose(conv.gradients()[0], gw, atol=1e-4)
    with pytest.raises(RuntimeError):
        conv.backward(torch.ones_like(ys[0]), 0)  # cache consumed


# --------------------------------------------------------------------------------- Dense
@pytest.mark.parametrize("cfg", [(1, 1, 1, True), (4, 12, 5, True), (8, 64, 10, False), (16, 200, 7, True),
                                 (3, 512, 200, True), (5, 7, 33, False)])
def test_dense_vs_autograd(cfg):
    N, In, Out, bias = cfg
    d = Dense(In, Out, bias, "d")
    d.set_seed(3)
    d.initialize()
    x = torch.randn(N, In, 1, 1)
    xr = x.view(N, In).clone().requires_grad_(True)
    wr = d.weights.detach().view(Out, In).clone().requires_grad_(True)
    br = d.bias.detach().view(-1).clone().requires_grad_(True) if bias else None
    ref = F.linear(xr, wr, br)
    y = d.forward(x)
    assert torch.allclose(y.view(N, Out), ref, atol=1e-5)
    dy = torch.randn(N, Out)
    ref.backward(dy)
    dx = d.backward(dy.view(N, Out, 1, 1))
    assert torch.allclose(dx.reshape(N, In), xr.grad, atol=1e-5)
    assert torch.allclose(d.gradients()[0].view(Out, In), wr.grad, atol=1e-5)
    if bias:
        assert torch.allclose(d.gradients()[1].view(-1), br.grad, atol=1e-5)
    assert d.forward_flops([N, In, 1, 1]) >= 2 * N * In * Out


def test_dense_flattens_nchw_in_reference_order():
    d = Dense(2 * 3 * 3, 4, True, "d")
    d.set_seed(5)
    d.initialize()
    x = torch.randn(2, 2, 3, 3)
    y = d.forward(x)
    ref = x.reshape(2, 18) @ d.weights.view(4, 18).t() + d.bias.view(-1)
    assert torch.allclose(y.view(2, 4), ref, atol=1e-5)


# --------------------------------------------------------------------------------- BatchNorm
@pytest.mark.parametrize("shape", [(2, 3, 4, 4), (8, 16, 2, 2), (4, 1, 5, 7), (16, 8, 1, 1), (3, 32, 6, 6)])
@pytest.mark.parametrize("affine", [True, False])
def test_batchnorm_train_vs_autograd(shape, affine):
    C = shape[1]
    bn = BatchNorm(C, 1e-5, 0.1, affine, "bn")
    bn.set_seed(1)
    bn.initialize()
    if affine:
        with torch.no_grad():
            bn.parameters()[0].uniform_(0.5, 1.5)
            bn.parameters()[1].uniform_(-0.5, 0.5)
    x = torch.randn(*shape) * 2 + 1
    xr = x.clone().requires_grad_(True)
    g = bn.parameters()[0].detach().view(-1).clone().requires_grad_(True) if affine else None
    b = bn.parameters()[1].detach().view(-1).clone().requires_grad_(True) if affine else None
    ref = F.batch_norm(xr, None, None, g, b, True, 0.1, 1e-5)
    y = bn.forward(x)
    assert torch.allclose(y, ref, atol=1e-4)
    dy = torch.randn_like(y)
    ref.backward(dy)
    dx = bn.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    if affine:
        assert torch.allclose(bn.gradients()[0].view(-1), g.grad, atol=1e-4)
        assert torch.allclose(bn.gradients()[1].view(-1), b.grad, atol=1e-4)
    # running stats: (1-m) r + m batch, unbiased variance
    n = x.numel() // C
    mean = x.mean((0, 2, 3))
    var = x.var((0, 2, 3), unbiased=False) * n / max(n - 1, 1)
    assert torch.allclose(bn.running_mean, 0.1 * mean, atol=1e-5)
    assert torch.allclose(bn.running_var, 0.9 + 0.1 * var, atol=1e-4)


@pytest.mark.parametrize("momentum", [0.1, 0.5, 1.0])
def test_batchnorm_eval_uses_running_stats(momentum):
    bn = BatchNorm(4, 1e-3, momentum, True, "bn")
    bn.initialize()
    x = torch.randn(8, 4, 3, 3) * 3 - 2
    bn.forward(x)
    bn.backward(torch.zeros(8, 4, 3, 3))
    bn.set_training(False)
    x2 = torch.randn(2, 4, 3, 3)
    y = bn.forward(x2)
    ref = (x2 - bn.running_mean.view(1, -1, 1, 1)) / torch.sqrt(bn.running_var.view(1, -1, 1, 1) + 1e-3)
    assert torch.allclose(y, ref, atol=1e-5)


def test_batchnorm_affine_grads_accumulate():
    """dgamma/dbeta accumulate across micro-batches (reference defect G4 overwrote on GPU)."""
    bn = BatchNorm(3, name="bn")
    bn.initialize()
    x = torch.randn(4, 3, 2, 2)
    dy = torch.randn(4, 3, 2, 2)
    bn.forward(x, 0)
    bn.forward(x, 1)
    bn.backward(dy, 0)
    g1 = bn.gradients()[0].clone()
    bn.backward(dy, 1)
    assert torch.allclose(bn.gradients()[0], 2 * g1, atol=1e-5)


def test_batchnorm_flops_and_config():
    bn = BatchNorm(16, 1e-3, 0.2, False, "bn")
    assert bn.forward_flops([2, 16, 4, 4]) == 6 * 2 * 16 * 16
    assert bn.backward_flops([2, 16, 4, 4]) == 9 * 2 * 16 * 16
    again = BatchNorm.from_config(bn.get_config())
    assert (again.epsilon, again.momentum, again.affine) == (1e-3, 0.2, False)
    assert bn.param_specs() == []


# --------------------------------------------------------------------------------- GroupNorm
@pytest.mark.parametrize("cfg", [(2, 8, 2, 4, 4), (1, 6, 3, 5, 5), (3, 16, 16, 2, 2), (2, 4, 1, 3, 3)])
def test_groupnorm_vs_autograd(cfg):
    N, C, G, H, W = cfg
    gn = GroupNorm(G, C, 1e-5, True, "gn")
    gn.initialize()
    with torch.no_grad():
        gn.parameters()[0].uniform_(0.5, 1.5)
        gn.parameters()[1].uniform_(-0.3, 0.3)
    x = torch.randn(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    g = gn.parameters()[0].detach().view(-1).clone().requires_grad_(True)
    b = gn.parameters()[1].detach().view(-1).clone().requires_grad_(True)
    ref = F.group_norm(xr, G, g, b, 1e-5)
    assert torch.allclose(gn.forward(x), ref, atol=1e-4)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    assert torch.allclose(gn.backward(dy), xr.grad, atol=1e-4)
    assert torch.allclose(gn.gradients()[0].view(-1), g.grad, atol=1e-4)
    assert torch.allclose(gn.gradients()[1].view(-1), b.grad, atol=1e-4)


def test_groupnorm_rejects_indivisible():
    with pytest.raises(ValueError):
        GroupNorm(3, 8)


# --------------------------------------------------------------------------------- pooling
POOL_CASES = [
    # N, C, H, W, ph, pw, sh, sw, pad_h, pad_w
    (1, 1, 4, 4, 2, 2, 2, 2, 0, 0), (2, 3, 8, 8, 2, 2, 2, 2, 0, 0), (2, 2, 7, 7, 3, 3, 2, 2, 1, 1),
    (1, 4, 9, 9, 3, 3, 3, 3, 0, 0), (2, 2, 6, 8, 2, 3, 2, 3, 0, 0), (1, 3, 5, 5, 3, 3, 1, 1, 1, 1),
    (2, 8, 4, 4, 4, 4, 4, 4, 0, 0), (1, 2, 6, 6, 2, 2, 1, 1, 0, 0), (3, 1, 10, 10, 3, 3, 2, 2, 0, 0),
]


@pytest.mark.parametrize("cfg", POOL_CASES)
def test_maxpool_vs_autograd(cfg):
    N, C, H, W, ph, pw, sh, sw, pdh, pdw = cfg
    mp = MaxPool2D(ph, pw, sh, sw, pdh, pdw, "mp")
    x = torch.randn(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, (ph, pw), (sh, sw), (pdh, pdw))
    y = mp.forward(x)
    assert torch.equal(y, ref)
    assert list(y.shape) == mp.compute_output_shape(list(x.shape))
    dy = torch.randn_like(ref)
    ref.backward(dy)
    assert torch.allclose(mp.backward(dy), xr.grad, atol=1e-6)


@pytest.mark.parametrize("cfg", POOL_CASES)
def test_avgpool_count_include_pad(cfg):
    """avg-pool divides by the full window even where it overlaps the padding
    (`src/nn/layers_impl/cuda/avgpool_ops.cu:53`)."""
    N, C, H, W, ph, pw, sh, sw, pdh, pdw = cfg
    ap = AvgPool2D(ph, pw, sh, sw, pdh, pdw, "ap")
    x = torch.randn(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    ref = F.avg_pool2d(xr, (ph, pw), (sh, sw), (pdh, pdw), count_include_pad=True)
    y = ap.forward(x)
    assert torch.allclose(y, ref, atol=1e-6)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    assert torch.allclose(ap.backward(dy), xr.grad, atol=1e-6)


def test_pool_default_strides():
    """LayerBuilder/layer default stride 0 -> pool size; SequentialBuilder defaults to stride 1
    (reference defect G10 kept for API compatibility)."""
    assert MaxPool2D(3, 3).stride_h == 3
    assert AvgPool2D(2, 2, 0, 0).stride_w == 2
    m = SequentialBuilder().input([1, 8, 8]).maxpool2d(2, 2).build()
    assert m.layers[0].stride_h == 1
    lb = LayerBuilder().input([1, 8, 8]).maxpool2d(2, 2).build()
    assert lb[0].stride_h == 2


# --------------------------------------------------------------------------------- activations, misc
@pytest.mark.parametrize("act", ["relu", "leaky_relu", "elu", "sigmoid", "tanh", "linear"])
@pytest.mark.parametrize("shape", [(2, 3, 4, 4), (5, 7, 1, 1)])
def test_activation_grad_vs_autograd(act, shape):
    a = Activation(act, "a")
    x = torch.randn(*shape)
    xr = x.clone().requires_grad_(True)
    fn = {"relu": F.relu, "leaky_relu": lambda t: F.leaky_relu(t, 0.01), "elu": F.elu, "sigmoid": torch.sigmoid,
          "tanh": torch.tanh, "linear": lambda t: t}[act]
    ref = fn(xr)
    assert torch.allclose(a.forward(x), ref, atol=1e-6)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    assert torch.allclose(a.backward(dy), xr.grad, atol=1e-5)


@pytest.mark.parametrize("p", [0.0, 0.25, 0.5])
def test_dropout_inverted_scaling_and_eval_identity(p):
    d = Dropout(p, "do")
    d.set_seed(3)
    x = torch.ones(64, 4, 8, 8)
    y = d.forward(x)
    kept = y != 0
    if p > 0:
        assert torch.allclose(y[kept], torch.full_like(y[kept], 1 / (1 - p)))
        assert abs(kept.float().mean().item() - (1 - p)) < 0.03
    g = d.backward(torch.ones_like(y))
    assert torch.equal(g != 0, kept)
    d.set_training(False)
    assert torch.equal(d.forward(x), x)


def test_flatten_roundtrip():
    f = Flatten("f")
    x = torch.randn(3, 4, 5, 6)
    y = f.forward(x)
    assert y.shape[0] == 3 and y.numel() == x.numel()
    assert torch.equal(f.backward(y).reshape(x.shape), x)


# --------------------------------------------------------------------------------- residual blocks
def _block_autograd(block, x, params):
    """Reference: the block's sub-layers composed from torch autograd ops, with the parameters
    taken in Sequential.parameters() order (main path, then shortcut) from ``params``."""
    it = iter(params)

    def run(path, t):
        for l in path:
            if isinstance(l, Conv2D):
                w = next(it)
                b = next(it).view(-1) if l.use_bias else None
                t = F.conv2d(t, w, b, (l.stride_h, l.stride_w), (l.pad_h, l.pad_w))
            elif isinstance(l, BatchNorm):
                g, b = next(it).view(-1), next(it).view(-1)
                t = F.batch_norm(t, None, None, g, b, True, 0.1, l.epsilon)
            elif isinstance(l, Activation):
                t = F.relu(t)
        return t
    h = run(block.main_path, x)
    s = run(block.shortcut_path, x) if block.shortcut_path else x
    return F.relu(h + s)


@pytest.mark.parametrize("cfg", [("basic", 8, 8, 1), ("basic", 8, 16, 2), ("basic", 4, 8, 1),
                                 ("bottleneck", 16, 16, 1), ("bottleneck", 8, 32, 2), ("bottleneck", 32, 32, 2)])
def test_residual_blocks_vs_autograd(cfg):
    kind, cin, cout, stride = cfg
    b = SequentialBuilder().input([cin, 8, 8])
    if kind == "basic":
        b.basic_residual_block(cin, cout, stride)
    else:
        b.bottleneck_residual_block(cin, max(cout // 4, 4), cout, stride)
    m = b.build()
    m.set_seed(4)
    m.initialize()
    m.set_first_layer_input_grad(True)
    blk = m.layers[0]
    assert isinstance(blk, ResidualBlock)
    assert bool(blk.shortcut_path) == (stride != 1 or cin != cout)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1 * torch.randn_like(p))  # BN affine away from (1, 0)
    params = [p.detach().clone().requires_grad_(True) for p in m.parameters()]
    x = torch.randn(2, cin, 8, 8)
    xr = x.clone().requires_grad_(True)
    ref = _block_autograd(blk, xr, params)
    y = m.forward(x)
    assert torch.allclose(y, ref, atol=1e-4)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    dx = m.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    for gg, r in zip(m.gradients(), params):
        assert torch.allclose(gg, r.grad, atol=2e-4)


def test_residual_config_roundtrip_json_string_paths():
    m = SequentialBuilder().input([8, 8, 8]).basic_residual_block(8, 16, 2).build()
    cfg = m.layers[0].get_config()
    assert isinstance(cfg.parameters["main_path"], str) and cfg.parameters["has_projection"]
    again = ResidualBlock.from_config(cfg)
    assert [l.type() for l in again.main_path] == [l.type() for l in m.layers[0].main_path]
    assert [l.type() for l in again.shortcut_path] == ["conv2d", "batchnorm"]


@pytest.mark.parametrize("name", ["resnet18_like", "resnet50_like"])
def test_sequential_resnet_like_architectures(name):
    """`sequential_residual_block_test.cpp` ResNet18/50-like stacks: shapes, parameter counts and
    finite gradients end to end."""
    b = SequentialBuilder().input([3, 32, 32]).conv2d(16, 3, 3, 1, 1, 1, 1, False).batchnorm().activation("relu")
    if name == "resnet18_like":
        b.basic_residual_block(16, 16, 1).basic_residual_block(16, 32, 2).basic_residual_block(32, 64, 2)
        final_c = 64
    else:
        b.bottleneck_residual_block(16, 8, 32, 1).bottleneck_residual_block(32, 16, 64, 2)
        b.bottleneck_residual_block(64, 32, 128, 2)
        final_c = 128
    m = b.avgpool2d(8, 8, 8, 8).flatten().dense(10).build()
    m.set_seed(9)
    m.initialize()
    assert m.compute_output_shape([4, 3, 32, 32]) == [4, 10, 1, 1]
    assert m.layers[-1].input_features == final_c
    out = m.forward(torch.randn(4, 3, 32, 32))
    assert out.shape == (4, 10, 1, 1) and torch.isfinite(out).all()
    m.backward(torch.randn_like(out))
    assert all(torch.isfinite(g).all() for g in m.gradients())
    assert m.num_parameters() == sum(p.numel() for p in m.parameters())


def test_layer_buffer_reuse_consistency():
    """Repeated forward/backward with the same input gives bit-identical results (no stale
    cached buffers), also when shapes change between calls (`layer_buffer_reuse_test.cpp`)."""
    m = SequentialBuilder().input([3, 8, 8]).conv2d(4, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu") \
        .maxpool2d(2, 2, 2, 2).flatten().dense(5).build()
    m.set_seed(1)
    m.initialize()
    x = torch.randn(2, 3, 8, 8)
    y1 = m.forward(x)
    m.backward(torch.ones_like(y1))
    g1 = [g.clone() for g in m.gradients()]
    m.clear_gradients()
    m.forward(torch.randn(5, 3, 8, 8))   # different batch in between
    m.backward(torch.ones(5, 5, 1, 1))
    m.clear_gradients()
    y2 = m.forward(x)
    m.backward(torch.ones_like(y2))
    assert torch.equal(y1, y2)
    for a, b in zip(g1, m.gradients()):
        assert torch.equal(a, b)


# --------------------------------------------------------------------------------- device manager
def test_device_manager_registry():
    from dcnn_amd.device import DeviceManager, DeviceType, get_cpu, get_device
    dm = DeviceManager.instance()
    assert DeviceManager.instance() is dm
    cpu = get_cpu()
    assert cpu.device_type == DeviceType.CPU and cpu.id == "CPU:0" and not cpu.is_gpu()
    assert get_device("cpu") is cpu and get_device(DeviceType.CPU) is cpu and get_device(torch.device("cpu")) is cpu
    assert "CPU:0" in dm.get_device_ids() and dm.has_device("cpu:0")
    n = torch.cuda.device_count()
    assert len(dm.get_devices_by_type(DeviceType.GPU)) == n
    for i in range(n):
        g = get_device(f"GPU:{i}")
        assert g.is_gpu() and g.id == f"GPU:{i}" and get_device(f"cuda:{i}") is g
    with pytest.raises(KeyError):
        get_device("GPU:99")
    with pytest.raises(RuntimeError):
        dm.get_gpu(99)
    dm.set_default_device("CPU")
    assert dm.get_default_device() is cpu


def test_device_alloc_copy_and_flow():
    from dcnn_amd.device import create_task, get_cpu
    cpu = get_cpu()
    t = cpu.allocate(10)
    assert t.numel() == 10 and t.device.type == "cpu"
    src = torch.arange(10, dtype=torch.float32)
    cpu.copy_to_device(t, src)
    assert torch.equal(t, src)
    task = create_task(cpu)
    task.sync()
    assert task.is_ready()
    assert cpu.get_total_memory() > 0


# --------------------------------------------------------------------------------- device agnosticity (GPU)
AGNOSTIC = [
    ("conv3x3", lambda b: b.conv2d(16, 3, 3, 1, 1, 1, 1)),
    ("conv3x3_s2", lambda b: b.conv2d(16, 3, 3, 2, 2, 1, 1)),
    ("conv1x1", lambda b: b.conv2d(24, 1, 1)),
    ("conv1x1_s2_nobias", lambda b: b.conv2d(16, 1, 1, 2, 2, 0, 0, False)),
    ("conv5x5_valid", lambda b: b.conv2d(8, 5, 5)),
    ("conv7x7_s2", lambda b: b.conv2d(16, 7, 7, 2, 2, 3, 3)),
    ("conv_bn_relu", lambda b: b.conv2d(16, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu")),
    ("conv_maxpool", lambda b: b.conv2d(16, 3, 3, 1, 1, 1, 1).maxpool2d(2, 2, 2, 2)),
    ("conv_dense", lambda b: b.conv2d(8, 3, 3, 2, 2, 1, 1).flatten().dense(10)),
    ("bn", lambda b: b.batchnorm()),
    ("groupnorm", lambda b: b.groupnorm(4)),
    ("maxpool3_s2_p1", lambda b: b.maxpool2d(3, 3, 2, 2, 1, 1)),
    ("avgpool2", lambda b: b.avgpool2d(2, 2, 2, 2)),
    ("avgpool_global", lambda b: b.avgpool2d(8, 8, 8, 8)),
    ("elu", lambda b: b.activation("elu")),
    ("sigmoid", lambda b: b.activation("sigmoid")),
    ("basic_block", lambda b: b.basic_residual_block(16, 16, 1)),
    ("basic_block_proj", lambda b: b.basic_residual_block(16, 32, 2)),
    ("bottleneck", lambda b: b.bottleneck_residual_block(16, 8, 32, 2)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", AGNOSTIC, ids=[c[0] for c in AGNOSTIC])
def test_device_agnosticity(case, dtype):
    """Same architecture and weights on CPU and on the GPU: forward, input gradient and every
    parameter gradient agree (fp32 GPU path tight; bf16 path within bf16 rounding)."""
    name, build = case
    torch.manual_seed(0)
    cpu = build(SequentialBuilder().input([16, 8, 8])).build()
    cpu.set_seed(21)
    cpu.initialize()
    gpu = build(SequentialBuilder().input([16, 8, 8])).build()
    gpu.set_seed(21)
    gpu.set_device("GPU:0")
    if dtype == "fp32":
        gpu.set_compute_dtype(torch.float32)
    gpu.initialize()
    gpu.load_parameters([p.clone() for p in cpu.parameters()])
    cpu.set_first_layer_input_grad(True)
    gpu.set_first_layer_input_grad(True)
    x = torch.randn(4, 16, 8, 8)
    yc = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    tol = 2e-4 if dtype == "fp32" else 3e-2
    assert _close(yg, yc, tol), (name, (yg.float().cpu() - yc).norm() / yc.norm())
    dy = torch.randn_like(yc)
    dxc = cpu.backward(dy)
    dxg = gpu.backward(dy.cuda())
    assert _close(dxg, dxc, 5 * tol), name
    gc = cpu.gradients()
    gg = gpu.gradients()
    scale = max([g.norm().item() for g in gc] + [1e-6])
    for a, b in zip(gc, gg):
        err = (b.float().cpu() - a).norm().item()
        assert err <= 5 * tol * max(a.norm().item(), 0.05 * scale) + 1e-6, (name, err, a.norm().item())
