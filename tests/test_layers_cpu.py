"""CPU layer tests against naive loop / autograd references (reference strategy:
`unit_tests/conv2d_layer_test.cpp:64-190`, `dense_layer_test.cpp`, `batchnorm_layer_test.cpp`,
`maxpool/avgpool tests`, `residual_block tests`)."""
import math

import pytest
import torch
import torch.nn.functional as F

from dcnn_amd.nn import (Activation, AvgPool2D, BatchNorm, Conv2D, Dense, Dropout, Flatten, GroupNorm, LayerBuilder,
                         MaxPool2D, ResidualBlock)


def naive_conv(x, w, b, s, p):
    N, C, H, W = x.shape
    Co, _, KH, KW = w.shape
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    xp = F.pad(x, (p, p, p, p))
    y = torch.zeros(N, Co, OH, OW, dtype=torch.float64)
    for oh in range(OH):
        for ow in range(OW):
            patch = xp[:, :, oh * s:oh * s + KH, ow * s:ow * s + KW].double()
            y[:, :, oh, ow] = torch.einsum("nchw,ochw->no", patch, w.double())
    if b is not None:
        y += b.double().view(1, -1, 1, 1)
    return y.float()


@pytest.mark.parametrize("cfg", [
    (1, 1, 5, 5, 1, 3, 1, 0), (2, 3, 8, 8, 4, 3, 1, 1), (2, 4, 9, 9, 6, 3, 2, 1), (1, 8, 6, 6, 16, 1, 1, 0),
    (2, 16, 8, 8, 8, 1, 2, 0), (1, 3, 14, 14, 8, 7, 2, 3), (2, 2, 7, 9, 3, 3, 1, 1),
])
def test_conv2d_forward_backward(cfg):
    N, C, H, W, Co, k, s, p = cfg
    conv = Conv2D(C, Co, k, k, s, s, p, p, True, "c")
    conv.set_seed(7)
    conv.initialize()
    x = torch.randn(N, C, H, W)
    y = conv.forward(x)
    ref = naive_conv(x, conv.weights, conv.bias.view(-1), s, p)
    assert torch.allclose(y, ref, atol=1e-4)
    # backward vs autograd; gradients accumulate
    dy = torch.randn_like(y)
    xr = x.clone().requires_grad_(True)
    wr = conv.weights.detach().clone().requires_grad_(True)
    br = conv.bias.detach().view(-1).clone().requires_grad_(True)
    F.conv2d(xr, wr, br, s, p).backward(dy)
    dx = conv.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    assert torch.allclose(conv.gradients()[0], wr.grad, atol=1e-4)
    assert torch.allclose(conv.gradients()[1].view(-1), br.grad, atol=1e-4)
    conv.forward(x, 3)
    conv.backward(dy, 3)
    assert torch.allclose(conv.gradients()[0], 2 * wr.grad, atol=1e-4)


def test_conv2d_init_kaiming_bound():
    conv = Conv2D(16, 32, 3, 3, name="c")
    conv.initialize()
    bound = 1 / math.sqrt(16 * 9)
    assert conv.weights.abs().max() <= bound + 1e-7
    assert conv.bias.abs().max() <= bound + 1e-7
    assert conv.weights.shape == (32, 16, 3, 3)


def test_dense():
    d = Dense(12, 5, True, "d")
    d.set_seed(1)
    d.initialize()
    x = torch.randn(4, 12, 1, 1)
    y = d.forward(x)
    ref = x.view(4, 12) @ d.weights.view(5, 12).t() + d.bias.view(-1)
    assert y.shape == (4, 5, 1, 1)
    assert torch.allclose(y.view(4, 5), ref, atol=1e-5)
    dy = torch.randn(4, 5, 1, 1)
    dx = d.backward(dy)
    assert torch.allclose(dx.view(4, 12), dy.view(4, 5) @ d.weights.view(5, 12), atol=1e-5)
    assert torch.allclose(d.gradients()[0].view(5, 12), dy.view(4, 5).t() @ x.view(4, 12), atol=1e-5)
    assert torch.allclose(d.gradients()[1].view(-1), dy.view(4, 5).sum(0), atol=1e-5)


def test_batchnorm_train_eval_and_grad():
    bn = BatchNorm(3, 1e-5, 0.1, True, "bn")
    bn.initialize()
    with torch.no_grad():
        bn.parameters()[0].copy_(torch.rand(3, 1, 1, 1) + 0.5)
        bn.parameters()[1].copy_(torch.randn(3, 1, 1, 1))
    x = torch.randn(4, 3, 5, 5) * 3 + 1
    y = bn.forward(x)
    g = bn.parameters()[0].view(-1).detach().clone().requires_grad_(True)
    b = bn.parameters()[1].view(-1).detach().clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    rm, rv = torch.zeros(3), torch.ones(3)
    ref = F.batch_norm(xr, rm, rv, g, b, True, 0.1, 1e-5)
    assert torch.allclose(y, ref, atol=1e-5)
    assert torch.allclose(bn.running_mean, rm, atol=1e-6)
    assert torch.allclose(bn.running_var, rv, atol=1e-5)  # unbiased running variance
    dy = torch.randn_like(y)
    ref.backward(dy)
    dx = bn.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    assert torch.allclose(bn.gradients()[0].view(-1), g.grad, atol=1e-4)
    assert torch.allclose(bn.gradients()[1].view(-1), b.grad, atol=1e-4)
    bn.set_training(False)
    ye = bn.forward(x)
    refe = F.batch_norm(x, rm, rv, g.detach(), b.detach(), False, 0.1, 1e-5)
    assert torch.allclose(ye, refe, atol=1e-5)


def test_groupnorm():
    gn = GroupNorm(2, 4, 1e-5, True, "gn")
    gn.initialize()
    with torch.no_grad():
        gn.parameters()[0].copy_(torch.rand(4, 1, 1, 1) + 0.5)
    x = torch.randn(3, 4, 5, 5)
    xr = x.clone().requires_grad_(True)
    g = gn.parameters()[0].view(-1).detach().clone().requires_grad_(True)
    b = gn.parameters()[1].view(-1).detach().clone().requires_grad_(True)
    ref = F.group_norm(xr, 2, g, b, 1e-5)
    y = gn.forward(x)
    assert torch.allclose(y, ref, atol=1e-5)
    dy = torch.randn_like(y)
    ref.backward(dy)
    dx = gn.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    assert torch.allclose(gn.gradients()[0].view(-1), g.grad, atol=1e-4)
    assert torch.allclose(gn.gradients()[1].view(-1), b.grad, atol=1e-4)


def test_pools():
    x = torch.randn(2, 3, 8, 8)
    mp = MaxPool2D(2, 2, 0, 0, 0, 0, "mp")  # stride 0 -> pool size
    assert mp.stride_h == 2
    y = mp.forward(x)
    assert torch.allclose(y, F.max_pool2d(x, 2))
    xr = x.clone().requires_grad_(True)
    F.max_pool2d(xr, 2).backward(torch.ones_like(y))
    assert torch.allclose(mp.backward(torch.ones_like(y)), xr.grad)
    ap = AvgPool2D(3, 3, 2, 2, 1, 1, "ap")
    y = ap.forward(x)
    assert torch.allclose(y, F.avg_pool2d(x, 3, 2, 1, count_include_pad=True), atol=1e-6)
    xr = x.clone().requires_grad_(True)
    F.avg_pool2d(xr, 3, 2, 1, count_include_pad=True).backward(torch.ones_like(y))
    assert torch.allclose(ap.backward(torch.ones_like(y)), xr.grad, atol=1e-6)


def test_maxpool_ties_first():
    x = torch.ones(1, 1, 2, 2)
    mp = MaxPool2D(2, 2, 2, 2, 0, 0, "mp")
    mp.forward(x)
    dx = mp.backward(torch.ones(1, 1, 1, 1))
    assert dx.view(-1).tolist() == [1.0, 0.0, 0.0, 0.0]


@pytest.mark.parametrize("act", ["relu", "leaky_relu", "elu", "sigmoid", "tanh", "linear", "softmax"])
def test_activation(act):
    a = Activation(act, "a")
    x = torch.randn(2, 5, 3, 3)
    xr = x.clone().requires_grad_(True)
    fn = {"relu": torch.relu, "leaky_relu": lambda t: F.leaky_relu(t, 0.01), "elu": F.elu, "sigmoid": torch.sigmoid,
          "tanh": torch.tanh, "linear": lambda t: t, "softmax": lambda t: torch.softmax(t, 1)}[act]
    ref = fn(xr)
    y = a.forward(x)
    assert torch.allclose(y, ref, atol=1e-6)
    dy = torch.randn_like(y)
    ref.backward(dy)
    assert torch.allclose(a.backward(dy), xr.grad, atol=1e-5)


def test_dropout_and_flatten():
    d = Dropout(0.5, "d")
    d.set_seed(3)
    x = torch.ones(1000)
    y = d.forward(x)
    assert set(torch.unique(y).tolist()) <= {0.0, 2.0}
    g = d.backward(torch.ones(1000))
    assert torch.equal(g, y)
    d.set_training(False)
    assert torch.equal(d.forward(x), x)
    f = Flatten("f")
    x = torch.randn(2, 3, 4, 5)
    y = f.forward(x)
    assert y.shape == (2, 60, 1, 1)
    assert torch.equal(y.view(2, 60), x.reshape(2, 60))
    assert torch.equal(f.backward(y), x)


def test_residual_block_matches_autograd():
    main = (LayerBuilder().input([4, 6, 6]).conv2d(8, 3, 3, 2, 2, 1, 1, True).batchnorm().activation("relu")
            .conv2d(8, 3, 3, 1, 1, 1, 1, True).batchnorm().build())
    short = LayerBuilder().input([4, 6, 6]).conv2d(8, 1, 1, 2, 2, 0, 0, False).batchnorm().build()
    blk = ResidualBlock(main, short, "relu", "rb")
    blk.set_seed(11)
    blk.initialize()
    x = torch.randn(2, 4, 6, 6)
    y = blk.forward(x)
    # autograd reference built from the same parameters
    c1, b1, _, c2, b2 = main
    sc, sb = short
    xr = x.clone().requires_grad_(True)
    ps = [p.detach().clone().requires_grad_(True) for p in blk.parameters()]

    def bnf(t, g, b):
        return F.batch_norm(t, None, None, g.view(-1), b.view(-1), True, 0.1, 1e-5)

    h = F.conv2d(xr, ps[0], ps[1].view(-1), 2, 1)
    h = torch.relu(bnf(h, ps[2], ps[3]))
    h = F.conv2d(h, ps[4], ps[5].view(-1), 1, 1)
    h = bnf(h, ps[6], ps[7])
    s = bnf(F.conv2d(xr, ps[8], None, 2, 0), ps[9], ps[10])
    ref = torch.relu(h + s)
    assert torch.allclose(y, ref, atol=1e-5)
    dy = torch.randn_like(y)
    ref.backward(dy)
    dx = blk.backward(dy)
    assert torch.allclose(dx, xr.grad, atol=1e-4)
    for g, p in zip(blk.gradients(), ps):
        assert torch.allclose(g, p.grad, atol=1e-4)


def test_layer_configs_roundtrip():
    from dcnn_amd.nn import LayerFactory
    layers = [Conv2D(3, 8, 3, 3, 1, 1, 1, 1, False, "c"), Dense(10, 4, True, "d"), BatchNorm(8, 1e-3, 0.2, True, "b"),
              GroupNorm(2, 8, 1e-5, True, "g"), MaxPool2D(3, 3, 2, 2, 1, 1, "m"), AvgPool2D(4, 4, 1, 1, 0, 0, "a"),
              Dropout(0.25, "dr"), Flatten("f"), Activation("elu", "e")]
    for l in layers:
        c = l.get_config()
        l2 = LayerFactory.create(l.type(), c)
        assert l2.get_config() == c
        assert l2.type() == l.type()
