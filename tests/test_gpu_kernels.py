"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op
(reference test strategy: `unit_tests/cuda_*_test.cpp`, `layer_device_agnosticity_test.cpp`).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from dcnn_amd.ops import fusion

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def rel_err(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def bf(x):
    return x.to(torch.bfloat16).float()


@pytest.fixture(scope="module")
def hip():
    from dcnn_amd.ops import hip as h
    from dcnn_amd.ops._ext import kernels
    assert kernels().arch == "gfx950"
    return h


CONV_CASES = [
    # N, Ci, H, W, Co, k, s, p
    (2, 32, 16, 16, 64, 3, 1, 1),
    (2, 64, 16, 16, 64, 3, 1, 1),
    (2, 64, 16, 16, 128, 3, 2, 1),
    (2, 64, 8, 8, 128, 1, 2, 0),
    (2, 3, 16, 16, 32, 3, 1, 1),
    (4, 512, 4, 4, 512, 3, 1, 1),
    (2, 128, 9, 9, 64, 3, 1, 1),
    (3, 64, 7, 5, 96, 3, 1, 1),
    (2, 256, 8, 8, 256, 1, 1, 0),
    (4, 32, 32, 32, 64, 3, 1, 1),   # dgrad: 32 output channels on the halo conv (half-filled tile)
    (2, 64, 16, 16, 32, 3, 1, 1),   # forward: 32 output channels on the halo conv
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(hip, case):
    N, Ci, H, W, Co, k, s, p = case
    torch.manual_seed(0)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, k, k) / math.sqrt(Ci * k * k)
    b = torch.randn(Co)
    xb, wb = bf(x), bf(w)
    y_ref = F.conv2d(xb, wb, b, s, p)
    xg = x.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    wg = w.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    y, partial = hip.conv2d_fwd(xg, wg, b.cuda(), (s, s), (p, p), stats=True)
    assert y.shape == y_ref.shape
    assert rel_err(y, y_ref) < 1e-2, rel_err(y, y_ref)
    # BN statistics from the epilogue
    stats = hip.bn_stats(y, partial)  # (mean, biased variance)
    yf = y.float().double()
    assert rel_err(stats[:Co], yf.mean((0, 2, 3))) < 1e-4
    assert rel_err(stats[Co:], yf.var((0, 2, 3), unbiased=False)) < 1e-4
    # dgrad
    dy = torch.randn_like(y_ref)
    dyb = bf(dy)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, wb, dyb, s, p)
    dyg = dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    wt = hip.conv_weight_t(wg)
    dx = hip.conv2d_dgrad(dyg, wt, x.shape, (s, s), (p, p))
    assert rel_err(dx, dx_ref) < 1e-2, rel_err(dx, dx_ref)
    # dgrad + fused residual
    r = torch.randn_like(x).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dx2 = hip.conv2d_dgrad(dyg, wt, x.shape, (s, s), (p, p), residual=r)
    assert rel_err(dx2, dx_ref + r.float().cpu()) < 1e-2
    # wgrad (accumulates into existing gradient) + bias grad
    gw = torch.ones(Co, Ci, k, k, device="cuda").contiguous(memory_format=CL)
    gb = torch.ones(Co, device="cuda")
    hip.conv2d_wgrad(dyg, xg, w.shape, (s, s), (p, p), gw, gb)
    dw_ref = torch.nn.grad.conv2d_weight(xb, w.shape, dyb, s, p) + 1
    assert rel_err(gw, dw_ref) < 1e-2, rel_err(gw, dw_ref)
    assert rel_err(gb, dyb.sum((0, 2, 3)) + 1) < 1e-2


def test_hconv_layer4_shape(hip):
    """Full ResNet layer-4 shape (4x4 maps, 512 channels, batch 256: 512 workgroups, 72 K steps
    each through the weight ring) of the halo conv, forward and dgrad, vs the fp32 reference."""
    N, C, H, W = 256, 512, 4, 4
    torch.manual_seed(4)
    x = torch.randn(N, C, H, W)
    w = torch.randn(C, C, 3, 3) / math.sqrt(C * 9)
    xg = x.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    wg = w.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    y, _ = hip.conv2d_fwd(xg, wg, None, (1, 1), (1, 1))
    assert rel_err(y, F.conv2d(bf(x), bf(w), None, 1, 1)) < 1e-2
    dy = torch.randn(N, C, H, W)
    dx = hip.conv2d_dgrad(dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL), hip.conv_weight_t(wg), x.shape,
                          (1, 1), (1, 1))
    assert rel_err(dx, torch.nn.grad.conv2d_input(x.shape, bf(w), bf(dy), 1, 1)) < 1e-2


@pytest.mark.parametrize("case", [
    # N, Ci, H, W, Co: halo-tiled wgrad geometries (TW=16 / 8 / 4, several images per tile)
    (4, 64, 32, 32, 64), (6, 128, 16, 16, 64), (4, 64, 16, 16, 192), (8, 256, 8, 8, 128), (16, 128, 4, 4, 256),
    (3, 64, 16, 48, 64),
])
@pytest.mark.parametrize("version", [2, 1])
def test_halo_wgrad(hip, case, version):
    """Both halo wgrad generations (2: tap-shift-invariant LDS addressing, 1: first kernel)."""
    from dcnn_amd.ops._ext import kernels
    kernels().hwgrad_set_version(version)
    try:
        _halo_wgrad_case(hip, case)
    finally:
        kernels().hwgrad_set_version(2)


@pytest.mark.parametrize("case", [(4, 32, 32, 32, 64), (6, 32, 16, 16, 128), (8, 32, 8, 8, 64), (16, 32, 4, 4, 64)])
def test_halo_wgrad_32_input_channels(hip, case):
    """Cs = 32 on the tap-shift-invariant halo wgrad (ResNet-18's first residual conv): one
    64-channel chunk whose upper half is read as zeros (buffer range) and never stored; every
    geometry against the fp32 reference, accumulating into the existing gradient. The first
    kernel generation does not take it."""
    from dcnn_amd.ops._ext import kernels
    N, Ci, H, W, Co = case
    kernels().hwgrad_set_version(1)
    try:
        assert not kernels().hwgrad_supported(N, H, W, Ci, Co, 9)
    finally:
        kernels().hwgrad_set_version(2)
    _halo_wgrad_case(hip, case)


def _halo_wgrad_case(hip, case):
    from dcnn_amd.ops._ext import kernels
    N, Ci, H, W, Co = case
    assert kernels().hwgrad_supported(N, H, W, Ci, Co, 9)
    torch.manual_seed(1)
    x = torch.randn(N, Ci, H, W)
    dy = torch.randn(N, Co, H, W)
    xg = x.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dyg = dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    gw = torch.full((Co, Ci, 3, 3), 0.5, device="cuda").contiguous(memory_format=CL)
    gb = torch.ones(Co, device="cuda")
    hip.conv2d_wgrad(dyg, xg, (Co, Ci, 3, 3), (1, 1), (1, 1), gw, gb)
    dw_ref = torch.nn.grad.conv2d_weight(bf(x), (Co, Ci, 3, 3), bf(dy), 1, 1) + 0.5
    assert rel_err(gw, dw_ref) < 1e-3, rel_err(gw, dw_ref)
    assert rel_err(gb, bf(dy).sum((0, 2, 3)) + 1) < 1e-4


def test_padded_rgb_stem(hip):
    """RGB stem runs on the vector path with channels zero-padded 3 -> 8."""
    torch.manual_seed(9)
    N, H, W, Co = 4, 20, 20, 32
    x = torch.randn(N, 3, H, W)
    w = torch.randn(Co, 3, 3, 3) / 5
    xp = hip.to_act_padded(x.cuda(), 8)
    assert xp.shape == (N, 8, H, W) and xp.is_contiguous(memory_format=CL)
    assert torch.equal(xp[:, 3:].float().cpu(), torch.zeros(N, 5, H, W))
    wp = hip.pad_weight_channels(w.cuda().bfloat16().contiguous(memory_format=CL), 8)
    y, _ = hip.conv2d_fwd(xp, wp, None, (1, 1), (1, 1))
    assert rel_err(y, F.conv2d(bf(x), bf(w), None, 1, 1)) < 1e-2
    dy = torch.randn(N, Co, H, W)
    gw = torch.zeros(Co, 3, 3, 3, device="cuda").contiguous(memory_format=CL)
    hip.conv2d_wgrad(dy.cuda().bfloat16().contiguous(memory_format=CL), xp, w.shape, (1, 1), (1, 1), gw)
    assert rel_err(gw, torch.nn.grad.conv2d_weight(bf(x), w.shape, bf(dy), 1, 1)) < 1e-2


@pytest.mark.parametrize("case", [
    # N, Ci, H, W, Co, bias, weight dtype/layout
    (4, 3, 64, 64, 32, False, "bf16_cl"), (3, 3, 32, 32, 64, True, "f32"), (2, 1, 32, 16, 16, True, "f32_cl"),
    (2, 4, 16, 128, 48, False, "bf16"),
])
def test_stem_conv(hip, case):
    """stem.hip: 3x3/s1/p1 conv straight from fp32 NCHW (fwd + BN statistics, wgrad + bias grad)
    against the fp32 reference on the bf16-rounded operands."""
    N, Ci, H, W, Co, use_b, wfmt = case
    torch.manual_seed(11)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, 3, 3) / math.sqrt(Ci * 9)
    b = torch.randn(Co) if use_b else None
    xg = x.cuda()
    assert hip.stem_ok(xg, w.shape, (1, 1), (1, 1))
    wg = w.cuda().to(torch.bfloat16 if wfmt.startswith("bf16") else torch.float32)
    if wfmt.endswith("_cl"):
        wg = wg.contiguous(memory_format=CL)
    y, partial = hip.stem_conv_fwd(xg, wg, b.cuda() if use_b else None, stats=True)
    y_ref = F.conv2d(bf(x), bf(w), b, 1, 1)
    assert y.shape == y_ref.shape and y.is_contiguous(memory_format=CL)
    assert rel_err(y, y_ref) < 1e-2, rel_err(y, y_ref)
    stats = hip.bn_stats(y, partial)  # (mean, biased variance)
    yf = y.float().double()
    assert rel_err(stats[:Co], yf.mean((0, 2, 3))) < 1e-4
    assert rel_err(stats[Co:], yf.var((0, 2, 3), unbiased=False)) < 1e-4
    dy = torch.randn(N, Co, H, W)
    dyg = dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    gw = torch.full((Co, Ci, 3, 3), 0.25, device="cuda")
    if wfmt.endswith("_cl"):
        gw = gw.contiguous(memory_format=CL)
    gb = torch.ones(Co, device="cuda") if use_b else None
    hip.stem_conv_wgrad(dyg, xg, gw, gb)
    dw_ref = torch.nn.grad.conv2d_weight(bf(x), w.shape, bf(dy), 1, 1) + 0.25
    assert rel_err(gw, dw_ref) < 1e-2, rel_err(gw, dw_ref)
    if use_b:
        assert rel_err(gb, bf(dy).sum((0, 2, 3)) + 1) < 1e-2


def test_multi_splitk_reduce(hip):
    """Batched split-K reduction (grad += sum over splits) over entries of every kind: float4 and
    scalar rows, 1 / several / > 32 splits (atomic groups), more entries than one launch holds."""
    from dcnn_amd.ops._ext import kernels
    torch.manual_seed(3)
    K = kernels()
    # 1-8 splits: one wave per chunk, 9-16: two, more: four (multi_splitk_reduce_kernel)
    shapes = [(1, 64), (5, 1000), (40, 36864), (100, 12), (33, 4608), (7, 3), (12, 500), (16, 4096), (256, 1024)] * 6
    slabs = [torch.randn(s, n, device="cuda") for s, n in shapes]
    outs = [torch.randn(n, device="cuda") for _, n in shapes]
    refs = [o.cpu() + sl.cpu().sum(0) for o, sl in zip(outs, slabs)]
    K.multi_splitk_reduce([(sl.data_ptr(), o.data_ptr(), o.numel(), sl.shape[0]) for sl, o in zip(slabs, outs)],
                          hip.stream_ptr())
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert rel_err(o, r) < 1e-5


def test_deferred_reduce_in_model_backward(hip):
    """Inside a model backward the wgrad reductions are queued and flushed by finish_backward:
    gradients read afterwards equal the per-layer immediate reduction (same model, same batch,
    conv layers run one by one outside any backward window)."""
    from dcnn_amd.models import create_model
    torch.manual_seed(8)
    m = create_model("mnist_cnn")
    m.set_seed(2)
    m.set_device("GPU:0")
    m.initialize()
    x = torch.randn(8, 1, 28, 28, device="cuda")
    out = m.forward(x, return_on_input_device=False)
    g = torch.randn_like(out.float())
    m.backward(g)
    assert not hip.grad_reducer.pending and not hip.grad_reducer.active
    deferred = [t.float().cpu().clone() for t in m.gradients()]
    m.clear_gradients()
    from dcnn_amd.ops import fusion
    prev = fusion.DEFER_REDUCE
    fusion.DEFER_REDUCE = False
    try:
        m.forward(x, return_on_input_device=False)
        m.backward(g)
    finally:
        fusion.DEFER_REDUCE = prev
    for a, b in zip(deferred, m.gradients()):
        assert rel_err(b, a) < 2e-2, rel_err(b, a)


@pytest.mark.parametrize("C", [32, 64, 8])
def test_bn_relu_maxpool(hip, C):
    """Fused training BatchNorm + ReLU + 2x2 max-pool == bn_apply(relu) then maxpool_fwd, bit for
    bit (pooled values, argmax, saved statistics, running statistics)."""
    torch.manual_seed(5)
    N, H, W = 4, 16, 12
    x = (torch.randn(N, C, H, W) * 2 + 0.5).cuda().bfloat16().contiguous(memory_format=CL)
    assert hip.bn_relu_maxpool_ok(x, 2, 2, 2, 2, 0, 0)
    gamma, beta = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    sums = hip.bn_stats(x, None)
    cnt = x.numel() // C
    m1, i1, m2, i2 = (torch.empty(C, device="cuda") for _ in range(4))
    r1 = (torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"))
    r2 = (torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"))
    yfull = hip.bn_apply(x, sums, cnt, gamma, beta, 1e-3, relu=True, save=(m1, i1), running=r1, momentum=0.1)
    y_ref, idx_ref = hip.maxpool_fwd(yfull, 2, 2, 2, 2, 0, 0)
    y, idx = hip.bn_relu_maxpool(x, sums, cnt, gamma, beta, 1e-3, (2, 2, 2, 2, 0, 0), save=(m2, i2), running=r2,
                                 momentum=0.1)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), y_ref.cpu())
    assert torch.equal(idx.cpu(), idx_ref.cpu())
    for a, b in [(m1, m2), (i1, i2), (r1[0], r2[0]), (r1[1], r2[1])]:
        assert torch.equal(a.cpu(), b.cpu())


@pytest.mark.parametrize("shape", [(128, 512, 200), (64, 256, 10), (16, 192, 10), (256, 1024, 200)])
def test_dense(hip, shape):
    N, In, Out = shape
    torch.manual_seed(1)
    x, w, b = torch.randn(N, In), torch.randn(Out, In) / math.sqrt(In), torch.randn(Out)
    y = hip.dense_fwd(x.cuda().bfloat16(), w.cuda().bfloat16(), b.cuda())
    assert rel_err(y, bf(x) @ bf(w).t() + b) < 1e-2
    dy = torch.randn(N, Out)
    wt = hip.conv_weight_t(w.cuda().bfloat16().view(Out, In, 1, 1)).view(In, Out)
    dx = hip.dense_dgrad(dy.cuda().bfloat16(), wt)
    assert rel_err(dx, bf(dy) @ bf(w)) < 1e-2
    gw = torch.zeros(Out, In, device="cuda")
    gb = torch.zeros(Out, device="cuda")
    hip.dense_wgrad(dy.cuda().bfloat16(), x.cuda().bfloat16(), gw, gb)
    assert rel_err(gw, bf(dy).t() @ bf(x)) < 1e-2
    assert rel_err(gb, bf(dy).sum(0)) < 1e-2


@pytest.mark.parametrize("C", [32, 64, 512, 12])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_batchnorm_fused(hip, C, dtype):
    torch.manual_seed(2)
    N, H, W = 4, 8, 8
    x = torch.randn(N, C, H, W) * 2 + 0.5
    g, bt = torch.rand(C) + 0.5, torch.randn(C)
    r = torch.randn(N, C, H, W)
    xg = x.cuda().to(dtype).contiguous(memory_format=CL)
    rg = r.cuda().to(dtype).contiguous(memory_format=CL)
    sums = hip.bn_stats(xg)
    mean = torch.empty(C, device="cuda")
    istd = torch.empty(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y = hip.bn_apply(xg, sums, N * H * W, g.cuda(), bt.cuda(), 1e-5, residual=rg, relu=True, save=(mean, istd),
                     running=(rm, rv), momentum=0.1)
    xf = xg.float().cpu()
    mu = xf.mean((0, 2, 3))
    var = xf.var((0, 2, 3), unbiased=False)
    ref = torch.relu((xf - mu.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + 1e-5) * g.view(1, -1, 1, 1)
                     + bt.view(1, -1, 1, 1) + rg.float().cpu())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert rel_err(y, ref) < tol
    assert rel_err(rm, 0.1 * mu) < 1e-3
    n = N * H * W
    assert rel_err(rv, 0.9 + 0.1 * var * n / (n - 1)) < 1e-3
    # backward with fused relu mask, accumulate dgamma/dbeta
    dy = torch.randn(N, C, H, W)
    dyg = dy.cuda().to(dtype).contiguous(memory_format=CL)
    dg, db = torch.ones(C, device="cuda"), torch.ones(C, device="cuda")
    dx, dmask = hip.bn_backward(dyg, xg, y, mean, istd, g.cuda(), dg, db, want_masked=True)
    xr = xf.clone().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = bt.clone().requires_grad_(True)
    out = torch.relu(F.batch_norm(xr, None, None, gr, br, True, 0.0, 1e-5) + rg.float().cpu())
    out.backward(dyg.float().cpu())
    assert rel_err(dx, xr.grad) < (3e-2 if dtype == torch.bfloat16 else 1e-3)
    assert rel_err(dg - 1, gr.grad) < 2e-2
    assert rel_err(db - 1, br.grad) < 2e-2
    assert rel_err(dmask, dyg.float().cpu() * (y.float().cpu() > 0)) < 1e-6


@pytest.mark.parametrize("case", [
    # N, C (BN channels = dgrad output), H, W, Co (dgrad input channels), stride, relu, residual
    (4, 64, 16, 16, 64, 1, True, False),     # hconv dgrad, ReLU mask
    (4, 64, 16, 16, 64, 1, True, True),      # + fused branch sum (ResNet block input gradient)
    (4, 64, 16, 16, 128, 2, True, True),     # strided: 4 phase-class g2 launches into one slab
    (2, 128, 8, 8, 64, 1, False, False),     # BN without a ReLU
    (8, 512, 4, 4, 512, 1, True, False),     # 4x4 layer-4 geometry
])
def test_dgrad_bwd_bn_fusion(hip, case):
    """conv dgrad with the consuming BatchNorm's ReLU mask + backward statistics in the epilogue
    (ops.hip.BnbRequest) == dgrad followed by the standalone BN backward."""
    N, C, H, W, Co, s, relu, resid = case
    torch.manual_seed(5)
    OH, OW = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    xb = (torch.randn(N, C, H, W) * 1.5 + 0.3).cuda().bfloat16().contiguous(memory_format=CL)
    g, bt = (torch.rand(C) + 0.5).cuda(), torch.randn(C).cuda()
    sums = hip.bn_stats(xb)
    mean, istd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    y = hip.bn_apply(xb, sums, N * H * W, g, bt, 1e-5, relu=relu, save=(mean, istd))
    yout = y if relu else None
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    dy = torch.randn(N, Co, OH, OW).cuda().bfloat16().contiguous(memory_format=CL)
    r = torch.randn(N, C, H, W).cuda().bfloat16().contiguous(memory_format=CL) if resid else None
    # unfused reference path
    d_ref = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (s, s), (1, 1), residual=r)
    dg0, db0 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx0, m0 = hip.bn_backward(d_ref, xb, yout, mean, istd, g, dg0, db0, want_masked=True)
    # fused
    req = hip.BnbRequest("bn", yout, xb, mean, istd)
    d = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (s, s), (1, 1), residual=r, bnb=req)
    assert getattr(d, "_bnb", None) is not None and d._bnb[0] == "bn"
    masked = d_ref.float() * (y.float() > 0) if relu else d_ref.float()
    assert rel_err(d, masked) < 1e-6
    dg1, db1 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx1, m1 = hip.bn_backward(d, xb, yout, mean, istd, g, dg1, db1, want_masked=True, fused=d._bnb[1:])
    assert rel_err(dx1, dx0) < 1e-2, rel_err(dx1, dx0)
    assert rel_err(dg1, dg0) < 1e-3, rel_err(dg1, dg0)
    assert rel_err(db1, db0) < 1e-3, rel_err(db1, db0)
    if relu:
        assert rel_err(m1, m0) < 1e-6


@pytest.mark.parametrize("C", [32, 64, 8])
def test_maxpool_bwd_bn_fusion(hip, C):
    """Stem pattern conv -> BN -> ReLU -> maxpool 2x2: the pool backward fused with the BN's ReLU
    mask (pooled value > 0) and backward statistics == pool backward + standalone BN backward."""
    torch.manual_seed(6)
    N, H, W = 4, 16, 16
    xb = (torch.randn(N, C, H, W) * 1.3 + 0.2).cuda().bfloat16().contiguous(memory_format=CL)
    g, bt = (torch.rand(C) + 0.5).cuda(), torch.randn(C).cuda()
    sums = hip.bn_stats(xb)
    mean, istd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    y = hip.bn_apply(xb, sums, N * H * W, g, bt, 1e-3, relu=True, save=(mean, istd))
    yp, idx = hip.maxpool_fwd(y, 2, 2, 2, 2, 0, 0)
    dyp = torch.randn(N, C, H // 2, W // 2).cuda().bfloat16().contiguous(memory_format=CL)
    d_ref = hip.maxpool_bwd(dyp, idx, (N, C, H, W), 2, 2, 2, 2, 0, 0)
    dg0, db0 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx0, _ = hip.bn_backward(d_ref, xb, y, mean, istd, g, dg0, db0)
    req = hip.BnbRequest("bn", y, xb, mean, istd)
    d = hip.maxpool_bwd(dyp, idx, (N, C, H, W), 2, 2, 2, 2, 0, 0, ypool=yp, bnb=req)
    assert getattr(d, "_bnb", None) is not None
    assert rel_err(d, d_ref.float() * (y.float() > 0)) < 1e-6
    dg1, db1 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx1, _ = hip.bn_backward(d, xb, y, mean, istd, g, dg1, db1, fused=d._bnb[1:])
    assert rel_err(dx1, dx0) < 1e-2, rel_err(dx1, dx0)
    assert rel_err(dg1, dg0) < 1e-3 and rel_err(db1, db0) < 1e-3


def test_pools_and_act(hip):
    torch.manual_seed(3)
    x = torch.randn(2, 32, 16, 16)
    xg = x.cuda().bfloat16().contiguous(memory_format=CL)
    xb = bf(x)
    for (ph, pw, sh, sw, pdh, pdw) in [(2, 2, 2, 2, 0, 0), (3, 3, 2, 2, 1, 1), (3, 3, 3, 3, 0, 0)]:
        y, idx = hip.maxpool_fwd(xg, ph, pw, sh, sw, pdh, pdw)
        yr, ir = F.max_pool2d(xb.requires_grad_(True), (ph, pw), (sh, sw), (pdh, pdw), return_indices=True)
        assert rel_err(y, yr) < 1e-6
        dy = torch.randn_like(yr)
        dx = hip.maxpool_bwd(dy.cuda().bfloat16().contiguous(memory_format=CL), idx, x.shape, ph, pw, sh, sw, pdh, pdw)
        xb.grad = None
        yr.backward(bf(dy))
        assert rel_err(dx, xb.grad) < 1e-2
        xb = bf(x)
        a = hip.avgpool_fwd(xg, ph, pw, sh, sw, pdh, pdw)
        ar = F.avg_pool2d(bf(x), (ph, pw), (sh, sw), (pdh, pdw), count_include_pad=True)
        assert rel_err(a, ar) < 1e-2
    # global average pool (4x4 -> 1x1) fwd/bwd
    x4 = torch.randn(3, 64, 4, 4)
    x4g = x4.cuda().bfloat16().contiguous(memory_format=CL)
    a = hip.avgpool_fwd(x4g, 4, 4, 1, 1, 0, 0)
    assert rel_err(a, bf(x4).mean((2, 3), keepdim=True)) < 1e-2
    d = hip.avgpool_bwd(torch.ones(3, 64, 1, 1, device="cuda", dtype=torch.bfloat16), x4.shape, 4, 4, 1, 1, 0, 0)
    assert torch.allclose(d.float(), torch.full_like(d.float(), 1 / 16))
    for kind in ["relu", "leaky_relu", "elu", "sigmoid", "tanh"]:
        from dcnn_amd.nn.activations import ActivationFactory
        fn = ActivationFactory.create(kind)
        xf = torch.randn(1000)
        yg = fn.apply(xf.cuda())
        assert rel_err(yg, fn.apply(xf)) < 1e-5
        gg = fn.gradient(xf.cuda(), yg, torch.ones(1000, device="cuda"))
        assert rel_err(gg, fn.gradient(xf, fn.apply(xf), torch.ones(1000))) < 1e-5
    s = hip.softmax_channels(xg)
    assert rel_err(s, torch.softmax(bf(x), 1)) < 1e-2


@pytest.mark.parametrize("kind", ["softmax_crossentropy", "logsoftmax_crossentropy", "crossentropy", "mse", "mae",
                                  "huber"])
def test_loss_fused(kind):
    from dcnn_amd.nn.loss import LossFactory
    torch.manual_seed(4)
    L = LossFactory.create(kind)
    p = torch.randn(64, 200, 1, 1)
    if kind == "crossentropy":
        p = torch.softmax(p, 1)
    lab = torch.randint(0, 200, (64,))
    t = F.one_hot(lab, 200).float().view(64, 200, 1, 1)
    lc, gc, cc = L.loss_and_grad(p, t)
    lg, gg, cg = L.loss_and_grad(p.cuda(), t.cuda())
    assert abs(lg.item() - lc.item()) < 1e-4 * max(1, abs(lc.item()))
    assert rel_err(gg, gc) < 1e-4
    assert cg.item() == cc.item()
    lg2, gg2, cg2 = L.loss_and_grad(p.cuda(), lab.cuda())
    assert abs(lg2.item() - lc.item()) < 1e-4 * max(1, abs(lc.item()))


def test_adam_sgd_flat():
    from dcnn_amd.nn.params import ParamArena, ParamSpec
    from dcnn_amd.nn.optimizers import SGD, Adam
    for make in [lambda: Adam(1e-2, weight_decay=0.01), lambda: Adam(1e-2, weight_decay=0.01, decouple_weight_decay=True),
                 lambda: SGD(0.1, 0.9), lambda: SGD(0.1)]:
        res = []
        for dev in ["cpu", "cuda"]:
            torch.manual_seed(5)
            specs = [ParamSpec("a", (7, 3, 3, 3), True), ParamSpec("b", (7, 1, 1, 1))]
            ar = ParamArena(specs, torch.device(dev), torch.bfloat16 if dev == "cuda" else None)
            ar.param(0).copy_(torch.randn(7, 3, 3, 3))
            ar.param(1).copy_(torch.randn(7, 1, 1, 1))
            ar.sync_shadow(force=True)
            opt = make()
            opt.attach([ar.param(0), ar.param(1)], [ar.grad_view(0), ar.grad_view(1)], ar)
            assert opt.arena is not None
            for it in range(3):
                ar.grad_view(0).copy_(torch.randn(7, 3, 3, 3))
                ar.grad_view(1).copy_(torch.randn(7, 1, 1, 1))
                opt.update()
            res.append((ar.param(0).cpu().clone(), ar))
        assert rel_err(res[1][0], res[0][0]) < 1e-5
        ar = res[1][1]
        assert rel_err(ar.shadow_view(0).float(), ar.param(0)) < 1e-2


def test_adam_reattach_restarts_device_step_counter():
    """An optimizer attached a second time restarts t, m, v: the device-side step counter and
    bias corrections must restart too, matching the host (CPU arena) update."""
    from dcnn_amd.nn.params import ParamArena, ParamSpec
    from dcnn_amd.nn.optimizers import Adam
    res = []
    for dev in ["cpu", "cuda"]:
        torch.manual_seed(7)
        ar = ParamArena([ParamSpec("a", (5, 4, 3, 3), True)], torch.device(dev),
                        torch.bfloat16 if dev == "cuda" else None)
        ar.param(0).copy_(torch.randn(5, 4, 3, 3))
        ar.sync_shadow(force=True)
        opt = Adam(1e-2)
        grads = [torch.randn(5, 4, 3, 3) for _ in range(5)]
        for attach_round in range(2):
            opt.attach([ar.param(0)], [ar.grad_view(0)], ar)
            for g in grads[:3] if attach_round == 0 else grads[3:]:
                ar.grad_view(0).copy_(g)
                opt.update()
        res.append(ar.param(0).cpu().clone())
    assert rel_err(res[1], res[0]) < 1e-5


def test_im2col_col2im(hip):
    x = torch.randn(2, 3, 7, 7)
    col = hip.im2col(x.cuda(), 3, 3, 2, 2, 1, 1)
    ref = F.unfold(x, 3, padding=1, stride=2)  # [N, C*9, L]
    ref = ref.permute(1, 0, 2).reshape(27, -1)
    assert rel_err(col, ref) < 1e-6
    back = hip.col2im(col, x.shape, 3, 3, 2, 2, 1, 1)
    ref2 = F.fold(F.unfold(x, 3, padding=1, stride=2), (7, 7), 3, padding=1, stride=2)
    assert rel_err(back, ref2) < 1e-6


def test_dropout_regenerates_mask(hip):
    x = torch.ones(10000, device="cuda")
    y = hip.dropout(x, 0.3, 1234)
    keep = (y > 0).float().mean().item()
    assert abs(keep - 0.7) < 0.03
    assert torch.allclose(y[y > 0], torch.full_like(y[y > 0], 1 / 0.7))
    g = hip.dropout(torch.ones(10000, device="cuda"), 0.3, 1234)
    assert torch.equal(g > 0, y > 0)


# ------------------------------------------------------------------ fp32 compute path (MFMA f32)
F32_CASES = CONV_CASES + [(2, 3, 32, 32, 64, 3, 1, 1), (2, 6, 9, 9, 10, 3, 2, 1), (1, 5, 7, 7, 7, 1, 1, 0),
                          (4, 64, 16, 16, 64, 3, 1, 1), (2, 128, 8, 8, 64, 3, 1, 1), (8, 64, 4, 4, 128, 3, 1, 1),
                          (2, 64, 32, 32, 128, 3, 1, 1),
                          # exact-fp32 halo conv: gutter layouts, split-K, a 16-channel input
                          (16, 64, 8, 8, 128, 3, 1, 1), (16, 128, 4, 4, 64, 3, 1, 1), (4, 16, 16, 16, 64, 3, 1, 1),
                          (64, 256, 8, 8, 256, 3, 1, 1),
                          # exact-fp32 halo wgrad: 32-channel blocks (not 64-multiples)
                          (4, 32, 16, 16, 96, 3, 1, 1), (8, 96, 4, 4, 32, 3, 1, 1)]


@pytest.fixture(params=["exact", "split", "concat"], ids=["f32exact", "f32split", "f32concat"])
def f32mode(request):
    """fp32 convs/GEMMs: exact v_mfma_f32_16x16x4_f32 gathered GEMMs; their split-precision 3xbf16
    variant; or (the default) 64-multiple 3x3 stride-1 convs on the bf16 halo kernels over
    [hi|lo|hi] channel concatenations (ops/hip.py _F32_CONCAT), the rest exact."""
    from dcnn_amd.ops import hip as H
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    prev, prev_c = K.get_f32_mode(), H.get_f32_concat()
    K.set_f32_mode(1 if request.param == "split" else 0)
    H.set_f32_concat(request.param == "concat")
    yield request.param
    K.set_f32_mode(prev)
    H.set_f32_concat(prev_c)


@pytest.mark.parametrize("case", F32_CASES)
def test_conv_fp32_fwd_dgrad_wgrad(hip, case, f32mode):
    N, Ci, H, W, Co, k, s, p = case
    torch.manual_seed(1)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, k, k) / math.sqrt(Ci * k * k)
    b = torch.randn(Co)
    xg = x.cuda().contiguous(memory_format=CL)
    wg = w.cuda().contiguous(memory_format=CL)
    r = torch.randn(F.conv2d(x, w, None, s, p).shape)
    h3 = dict(hip._H3_F32_STATS)
    y, partial = hip.conv2d_fwd(xg, wg, b.cuda(), (s, s), (p, p), stats=True,
                                residual=r.cuda().contiguous(memory_format=CL), relu=True)
    y_ref = torch.relu(F.conv2d(x, w, b, s, p) + r)
    assert y.dtype == torch.float32
    concat = (f32mode == "concat" and Ci % 64 == 0 and Co % 64 == 0 and k == 3 and s == 1 and p == 1
              and hip.kernels().hconv_supported(N, H, W, 3 * Ci, Co, 9))
    assert hasattr(xg, "_s3") == concat  # the split-precision halo path ran exactly when eligible
    h3_ok = (not concat and k == 3 and s == 1 and p == 1 and hip.kernels().hconv3_f32_splits(N, H, W, Ci, Co, 9) > 0)
    assert (hip._H3_F32_STATS["fwd"] > h3["fwd"]) == h3_ok  # the exact fp32 halo conv ran exactly when eligible
    assert rel_err(y, y_ref) < 1e-5, rel_err(y, y_ref)
    stats = hip.bn_stats(y, partial)  # (mean, biased variance)
    assert rel_err(stats[:Co], y_ref.double().mean((0, 2, 3))) < 1e-5
    assert rel_err(stats[Co:], y_ref.double().var((0, 2, 3), unbiased=False)) < 1e-5
    dy = torch.randn_like(y_ref)
    dyg = dy.cuda().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(wg, dtype=torch.float32)
    dx = hip.conv2d_dgrad(dyg, wt, x.shape, (s, s), (p, p))
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, s, p)
    assert dx.dtype == torch.float32 and rel_err(dx, dx_ref) < 1e-5, rel_err(dx, dx_ref)
    gw = torch.ones(Co, Ci, k, k, device="cuda").contiguous(memory_format=CL)
    gb = torch.ones(Co, device="cuda")
    h3 = dict(hip._H3_F32_STATS)
    hip.conv2d_wgrad(dyg, xg, w.shape, (s, s), (p, p), gw, gb)
    hw_ok = not concat and k == 3 and s == 1 and p == 1 and hip.kernels().hwgrad_f32_supported(N, H, W, Ci, Co)
    assert (hip._H3_F32_STATS["wgrad"] > h3["wgrad"]) == hw_ok  # the exact fp32 halo wgrad ran when eligible
    gw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, s, p) + 1
    assert rel_err(gw, gw_ref) < 1e-5, rel_err(gw, gw_ref)
    assert rel_err(gb, dy.sum((0, 2, 3)) + 1) < 1e-5


@pytest.mark.parametrize("shape", [(8, 512, 200), (5, 27, 10), (64, 256, 128)])
def test_dense_fp32(hip, shape, f32mode):
    N, In, Out = shape
    torch.manual_seed(2)
    x, w, b = torch.randn(N, In), torch.randn(Out, In) / math.sqrt(In), torch.randn(Out)
    y = hip.dense_fwd(x.cuda(), w.cuda(), b.cuda())
    assert rel_err(y, x @ w.t() + b) < 1e-5
    dy = torch.randn(N, Out)
    wt = hip.conv_weight_t(w.cuda().view(Out, In, 1, 1), dtype=torch.float32).view(In, Out)
    assert rel_err(hip.dense_dgrad(dy.cuda(), wt), dy @ w) < 1e-5
    gw, gb = torch.zeros(Out, In, device="cuda"), torch.zeros(Out, device="cuda")
    hip.dense_wgrad(dy.cuda(), x.cuda(), gw, gb)
    assert rel_err(gw, dy.t() @ x) < 1e-5 and rel_err(gb, dy.sum(0)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_stats_large_mean_matches_fp64(hip, dtype):
    """mean 1e3, std 1: E[x^2] - mean^2 in fp32 would lose every digit of the variance; the
    pivot-shifted tile statistics + Chan merges match the fp64 variance to 1e-3 (16384 rows:
    the two-level ticketed reduce runs)."""
    torch.manual_seed(11)
    N, C, H, W = 64, 64, 16, 16
    x = (1e3 + torch.randn(N, C, H, W)).cuda().to(dtype).contiguous(memory_format=CL)
    assert hip.kernels().bn_stat_parts(hip.kernels().bn_partial_rows(N * H * W, C)) > 1
    st = hip.bn_stats(x)
    xd = x.double()
    assert rel_err(st[:C], xd.mean((0, 2, 3))) < 1e-6
    var = xd.var((0, 2, 3), unbiased=False)
    assert ((st[C:].double().cpu() - var.cpu()).abs() / var.cpu()).max() < 1e-3


@pytest.mark.parametrize("shape", [(8, 64, 32, 32, 64), (16, 64, 8, 8, 128), (8, 24, 12, 12, 40), (8, 3, 12, 12, 20)])
def test_conv_epilogue_stats_large_mean_and_deterministic(hip, shape):
    """Conv-epilogue BatchNorm statistics (hconv / gemm_g2 / v1 paths) with a 1e3 bias: variance
    matches fp64 of the stored output to 1e-3, and two runs are bit-identical."""
    N, Ci, H, W, Co = shape
    torch.manual_seed(12)
    x = torch.randn(N, Ci, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(Co, Ci, 3, 3) / math.sqrt(9 * Ci)).cuda().bfloat16().contiguous(memory_format=CL)
    b = torch.full((Co,), 1e3, device="cuda")
    outs = []
    for _ in range(2):
        y, partial = hip.conv2d_fwd(x, w, b, (1, 1), (1, 1), stats=True)
        outs.append((y, hip.bn_stats(y, partial).clone()))
    (y, st), (y2, st2) = outs
    assert torch.equal(y, y2) and torch.equal(st, st2)
    yd = y.double()
    var = yd.var((0, 2, 3), unbiased=False).cpu()
    assert rel_err(st[:Co], yd.mean((0, 2, 3))) < 1e-6
    assert ((st[Co:].double().cpu() - var).abs() / var).max() < 1e-3


def test_stat_reduce_many_rows_deterministic(hip):
    """bn_stat_reduce with several hundred slab rows in both modes: equals an fp64 reference and
    is bit-identical across runs (fixed-order partials, merged in part order by the consumer)."""
    torch.manual_seed(13)
    rows, C = 1000, 200
    n = torch.randint(1, 50, (rows, 1)).float().expand(rows, C)
    mean = torch.randn(rows, C) * 3 + 7
    m2 = torch.rand(rows, C) * n
    slab = torch.stack([n, mean, m2], 1).contiguous().cuda()
    out = [hip.stat_reduce(0, slab, rows, C, torch.empty(2 * C, device="cuda")).clone() for _ in range(2)]
    assert torch.equal(out[0], out[1])
    nd, md, m2d = n.double(), mean.double(), m2.double()
    tot = nd.sum(0)
    mu = (nd * md).sum(0) / tot
    var = (m2d.sum(0) + (nd * (md - mu) ** 2).sum(0)) / tot
    assert rel_err(out[0][:C], mu) < 1e-6 and rel_err(out[0][C:], var) < 1e-5
    slab1 = torch.randn(rows, 2, C).cuda()
    s1 = [hip.stat_reduce(1, slab1, rows, C, torch.empty(2 * C, device="cuda")).clone() for _ in range(2)]
    assert torch.equal(s1[0], s1[1])
    ref = slab1.double().sum(0).reshape(-1).cpu()
    assert (s1[0].double().cpu() - ref).abs().max() < 1e-4


def test_fp32_split_precision_error_bound(hip):
    """The 3xbf16 split GEMM and the split-precision halo conv ([hi|lo|hi] channel concatenation)
    against an fp64 reference on a deep reduction (K = 4608, the ResNet layer-4 conv): relative
    error <= 1e-5 in norm and close to the exact f32 MFMA's."""
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    prev, prev_c = K.get_f32_mode(), hip.get_f32_concat()
    torch.manual_seed(7)
    x = torch.randn(8, 512, 8, 8)
    w = torch.randn(256, 512, 3, 3) / math.sqrt(512 * 9)
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    errs = {}
    try:
        for mode in ("exact", "split", "concat"):
            K.set_f32_mode(1 if mode == "split" else 0)
            hip.set_f32_concat(mode == "concat")
            y, _ = hip.conv2d_fwd(x.cuda().contiguous(memory_format=CL), w.cuda().contiguous(memory_format=CL),
                                  None, (1, 1), (1, 1))
            errs[mode] = ((y.double().cpu() - ref).norm() / ref.norm()).item()
    finally:
        K.set_f32_mode(prev)
        hip.set_f32_concat(prev_c)
    print(errs)
    assert errs["split"] < 1e-5 and errs["concat"] < 1e-5, errs
    assert errs["exact"] < 3e-6, errs


def test_split3_rows(hip):
    """fp32 -> [hi|lo|hi] / [hi|hi|lo] bf16 rows: hi is the bf16 rounding, hi + lo within 2^-16."""
    torch.manual_seed(8)
    x = (torch.randn(37, 64) * 10).cuda()
    for pattern in (0, 1):
        s = hip.split3_rows(x, 37, 64, pattern).float()
        hi = x.bfloat16().float()
        lo = s[:, 64:128] if pattern == 0 else s[:, 128:]
        assert torch.equal(s[:, :64], hi)
        assert torch.equal(s[:, 128:] if pattern == 0 else s[:, 64:128], hi)
        assert ((hi + lo - x).abs() <= x.abs() * 2.0 ** -16 + 1e-30).all()


@pytest.mark.parametrize("case", [(4, 512, 4, 4, 512), (16, 256, 8, 8, 256), (8, 128, 16, 16, 128)])
def test_hconv_split_k_matches_unsplit(hip, case):
    """Split-K halo conv (small grids: partial tiles summed in split order by the last workgroup
    of each tile) vs the unsplit kernel and the fp32 reference, forward + stats and dgrad;
    repeated launches are bit-identical (ticket words left zeroed)."""
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    N, C, H, W, Co = case
    assert K.hconv_splits(N, H, W, C, Co, 9) > 1
    torch.manual_seed(3)
    x = torch.randn(N, C, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(Co).cuda()
    dy = torch.randn(N, Co, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    outs = []
    prev = K.hconv_split_target()
    try:
        for target in (512, 512, 0):
            K.hconv_set_split_target(target)
            y, part = hip.conv2d_fwd(x, w, b, (1, 1), (1, 1), stats=True, relu=True)
            st = hip.bn_stats(y, part)
            dx = hip.conv2d_dgrad(dy, wt, x.shape, (1, 1), (1, 1))
            outs.append((y.clone(), st.clone(), dx.clone()))
    finally:
        K.hconv_set_split_target(prev)
    (y1, s1, d1), (y2, s2, d2), (y0, s0, d0) = outs
    assert torch.equal(y1, y2) and torch.equal(s1, s2) and torch.equal(d1, d2)
    ref = F.relu(F.conv2d(x.float().cpu(), w.float().cpu(), b.cpu(), 1, 1))
    assert rel_err(y1, ref) < 1e-2 and rel_err(y0, ref) < 1e-2
    assert rel_err(y1, y0) < 5e-3 and rel_err(d1, d0) < 5e-3
    assert rel_err(s1, s0) < 1e-3


@pytest.mark.parametrize("case", [(4, 128, 8, 8, 128), (2, 512, 4, 4, 256), (8, 256, 8, 8, 512), (8, 512, 8, 8, 256),
                                  (8, 256, 8, 8, 256), (8, 128, 16, 16, 128), (8, 128, 16, 16, 256), (8, 512, 4, 4, 512)])
def test_hconv_fp32_concat_accuracy(hip, case):
    """fp32 split-precision halo conv (fp32 epilogue) vs fp64 on the ResNet-9 batch-8 shapes,
    under both split-K targets (the fp32 convs stay unsplit: ops/hip.py _NOSPLIT)."""
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    N, C, H, W, Co = case
    torch.manual_seed(4)
    x = torch.randn(N, C, H, W, dtype=torch.float64)
    w = torch.randn(Co, C, 3, 3, dtype=torch.float64) / math.sqrt(9 * C)
    ref = F.conv2d(x, w, None, 1, 1)
    dy = torch.randn(N, Co, H, W, dtype=torch.float64)
    dref = torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 1)
    xg = x.float().cuda().contiguous(memory_format=CL)
    wg = w.float().cuda().contiguous(memory_format=CL)
    dyg = dy.float().cuda().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(wg, dtype=torch.float32)
    res = []
    prev = K.hconv_split_target()
    try:
        for target in (512, 0):
            K.hconv_set_split_target(target)
            y, _ = hip.conv2d_fwd(xg, wg, None, (1, 1), (1, 1))
            dx = hip.conv2d_dgrad(dyg, wt, x.shape, (1, 1), (1, 1))
            res.append((y, dx))
    finally:
        K.hconv_set_split_target(prev)
    for y, dx in res:
        assert rel_err(y.double(), ref) < 2e-5, rel_err(y.double(), ref)
        assert rel_err(dx.double(), dref) < 2e-5, rel_err(dx.double(), dref)
    # element-wise: no output of the split kernel further from fp64 than the unsplit one's worst
    for a, b, r in ((res[0][0], res[1][0], ref), (res[0][1], res[1][1], dref)):
        ea = (a.double().cpu() - r).abs().max().item()
        eb = (b.double().cpu() - r).abs().max().item()
        assert ea < 4 * eb + 1e-7, (ea, eb)


@pytest.mark.parametrize("case", [(8, 64, 32, 32, 128), (16, 128, 16, 16, 256), (16, 256, 8, 8, 512), (4, 64, 64, 64, 64),
                                  (32, 128, 32, 32, 128)])
@pytest.mark.parametrize("bias", [False, True])
def test_wgrad_stride2_halo(hip, case, bias, monkeypatch):
    """3x3 stride-2 weight gradient on the stride-2 halo kernel (hwgrad_s2: 64-pixel tiles, the
    input halo staged once for all taps) == the gathered gemm_t2 path and the fp32 reference
    (weights and bias accumulate into the existing gradient: beta = 1)."""
    from dcnn_amd.ops._ext import kernels
    N, Ci, H, W, Co = case
    assert kernels().hwgrad_s2_supported(N, H // 2, W // 2, Ci, Co)
    torch.manual_seed(10)
    x = torch.randn(N, Ci, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, Co, H // 2, W // 2).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    g0 = torch.randn(Co, Ci, 3, 3).cuda().contiguous(memory_format=CL)
    outs = []
    for s2 in (True, False):
        monkeypatch.setattr(fusion, "HWGRAD_S2", s2)
        gw = g0.clone()
        gb = torch.ones(Co, device="cuda") if bias else None
        hip.conv2d_wgrad(dy, x, (Co, Ci, 3, 3), (2, 2), (1, 1), gw, gb)
        outs.append((gw, gb))
    ref = torch.nn.grad.conv2d_weight(x.float().cpu(), (Co, Ci, 3, 3), dy.float().cpu(), 2, 1) + g0.cpu()
    for gw, gb in outs:
        assert rel_err(gw, ref) < 1e-4, rel_err(gw, ref)
        if bias:
            assert rel_err(gb, dy.float().sum((0, 2, 3)) + 1) < 1e-4
    assert rel_err(outs[0][0], outs[1][0]) < 1e-4


@pytest.mark.parametrize("case", [(8, 64, 32, 32, 128, 3, 2, 1), (16, 256, 8, 8, 512, 3, 2, 1), (4, 32, 16, 16, 64, 5, 2, 2),
                                  (8, 64, 16, 16, 128, 1, 2, 0), (16, 256, 8, 8, 512, 1, 2, 0)])
def test_strided_dgrad_grouped_launch(hip, case, monkeypatch):
    """All stride phases of a strided dgrad in one grouped gemm_g2 launch == one launch per phase
    (bit-identical: same per-row K order), with residual and the fused backward-BN request."""
    N, Ci, H, W, Co, k, s, p = case
    torch.manual_seed(7)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    w = (torch.randn(Co, Ci, k, k) / math.sqrt(Ci * k * k)).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, Co, OH, OW).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    res = torch.randn(N, Ci, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    outs = []
    for grouped in (True, False):
        monkeypatch.setattr(fusion, "G2_GROUP", grouped)
        outs.append(hip.conv2d_dgrad(dy, wt, (N, Ci, H, W), (s, s), (p, p), residual=res))
    assert torch.equal(outs[0], outs[1])
    ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w.float().cpu(), dy.float().cpu(), s, p) + res.float().cpu()
    assert rel_err(outs[0], ref) < 1e-2


@pytest.mark.parametrize("relu", [False, True])
def test_bn_backward_eval_mode_kernels(hip, relu):
    """Frozen-statistics (eval-mode) BatchNorm backward: dx = gamma * istd * dy' and the affine
    gradients, all on the HIP kernels (bn_partial + bn_bwd_apply), vs fp32 reference math."""
    torch.manual_seed(8)
    N, C, H, W = 4, 64, 8, 8
    x = torch.randn(N, C, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, C, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    rm, rv = torch.randn(C).cuda() * 0.1, torch.rand(C).cuda() + 0.5
    istd = 1.0 / (rv + 1e-5).sqrt()
    gamma = torch.randn(C).cuda()
    yout = torch.relu(x) if relu else None
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx, dmask = hip.bn_backward(dy, x, yout, rm, istd, gamma, dg, db, want_masked=True, eval_mode=True)
    d = dy.float() * ((yout.float() > 0).float() if relu else 1.0)
    xhat = (x.float() - rm.view(1, -1, 1, 1)) * istd.view(1, -1, 1, 1)
    assert rel_err(dx, d * (gamma * istd).view(1, -1, 1, 1)) < 1e-2
    assert rel_err(dg, (d * xhat).sum((0, 2, 3))) < 1e-4
    assert rel_err(db, d.sum((0, 2, 3))) < 1e-4
    if relu:
        assert rel_err(dmask, d) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
@pytest.mark.parametrize("shape", [(256, 64, 32, 32), (64, 128, 16, 16), (32, 256, 8, 8), (16, 512, 4, 4), (3, 24, 5, 7)])
def test_bn_apply_vectorised_matches_generic(hip, shape, dtype):
    """Vectorised BatchNorm apply passes (bn_apply_v / bn_bwd_apply_v: 8-element vectors, U = 1 / 2
    / 4 per lane by size, statistics prologue behind the first loads; bf16 and fp32) == the generic
    kernels: forward (+residual, ReLU, running statistics) bit-identical; backward (3-coefficient
    form, ReLU mask) within rounding; dgamma / dbeta identical."""
    from dcnn_amd.ops._ext import kernels
    K = kernels()
    N, C, H, W = shape
    torch.manual_seed(11)
    mk = lambda: torch.randn(N, C, H, W).cuda().to(dtype).contiguous(memory_format=CL)
    x, r, dy, yo = mk(), mk(), mk(), mk()
    R = N * H * W
    parts = 3
    part = torch.empty(parts, 3, C, device="cuda")
    part[:, 0] = R / parts
    part[:, 1] = torch.randn(parts, C, device="cuda") * 0.2
    part[:, 2] = (R / parts) * (0.5 + torch.rand(parts, C, device="cuda"))
    stats = hip.Stats(part, parts, 0)
    g, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    mean, istd = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    sums = torch.randn(2 * C, device="cuda") * R * 0.01
    outs = []
    try:
        for vec in (1, 0):
            K.bn_set_vectorised(vec)
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            sm, si = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
            y1 = hip.bn_apply(x, stats, R, g, b, 1e-5, relu=True, save=(sm, si), running=(rm, rv))
            y2 = hip.bn_apply(x, stats, R, g, b, 1e-5, residual=r, relu=True)
            res = []
            for mask in (0, 1):
                dx = torch.empty_like(x)
                dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
                K.bn_bwd_apply(int(dtype == torch.bfloat16), dy.data_ptr(), yo.data_ptr() if mask else 0, x.data_ptr(),
                               dx.data_ptr(), R, C,
                               mean.data_ptr(), istd.data_ptr(), g.data_ptr(), sums.data_ptr(), 1, float(R),
                               dg.data_ptr(), db.data_ptr(), 0, hip.stream_ptr())
                res.append((dx, dg, db))
            torch.cuda.synchronize()
            outs.append((y1, y2, rm, rv, sm, si, res))
    finally:
        K.bn_set_vectorised(1)
    (a1, a2, arm, arv, asm, asi, ares), (b1, b2, brm, brv, bsm, bsi, bres) = outs
    assert torch.equal(a1, b1) and torch.equal(a2, b2)
    for u, v in ((arm, brm), (arv, brv), (asm, bsm), (asi, bsi)):
        assert torch.equal(u, v)
    for (dxa, dga, dba), (dxb, dgb, dbb) in zip(ares, bres):
        assert torch.equal(dga, dgb) and torch.equal(dba, dbb)
        tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
        assert (dxa.float() - dxb.float()).abs().max().item() <= tol * dxb.float().abs().max().item()


@pytest.mark.parametrize("geom", [(3, 3, 2, 2, 1, 1), (2, 2, 2, 2, 0, 0), (3, 3, 1, 1, 1, 1)])
def test_maxpool_vectorised_vs_torch(hip, geom):
    """bf16 max-pool forward / backward on the 8-channel vector kernels (overlapping windows: the
    ResNet-50 stem 3x3 / s2 / p1) against torch.nn.functional.max_pool2d. Inputs are distinct bf16
    values, so the argmax is unique: pooled values match exactly, gradients to bf16 rounding."""
    ph, pw, sh, sw, pad_h, pad_w = geom
    N, C, H, W = 1, 64, 18, 18
    torch.manual_seed(21)
    n = N * C * H * W
    # n distinct finite bf16 values (consecutive positive bit patterns), shuffled, random signs
    bits = (torch.arange(n, dtype=torch.int32) + 0x0800)[torch.randperm(n)]
    vals = bits.to(torch.int16).view(torch.bfloat16).float()
    vals = torch.where(torch.rand(n) < 0.5, -vals, vals)
    x = vals.view(N, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, (ph, pw), (sh, sw), (pad_h, pad_w))
    dy = torch.randn_like(yr).bfloat16().float()
    yr.backward(dy)
    xg = x.cuda().bfloat16().contiguous(memory_format=CL)
    y, idx = hip.maxpool_fwd(xg, ph, pw, sh, sw, pad_h, pad_w)
    assert torch.equal(y.float().cpu(), yr.detach().bfloat16().float())
    dx = hip.maxpool_bwd(dy.cuda().bfloat16().contiguous(memory_format=CL), idx, (N, C, H, W), ph, pw, sh, sw, pad_h,
                         pad_w)
    assert rel_err(dx, xr.grad) < 1e-2  # bf16 rounding of summed window gradients only


@pytest.mark.parametrize("geom", [(2, 2, 2, 2, 0, 0), (3, 3, 3, 3, 0, 0), (3, 3, 2, 2, 1, 1)])
@pytest.mark.parametrize("C", [12, 64])
def test_maxpool_fp32_vs_torch(hip, geom, C):
    """fp32 max-pool forward / backward (the 4-channel vector kernels on non-overlapping windows,
    the generic kernel otherwise) against torch.nn.functional.max_pool2d: distinct values, so the
    argmax is unique and both directions match exactly."""
    ph, pw, sh, sw, pad_h, pad_w = geom
    N, H, W = 2, 18, 18
    torch.manual_seed(22)
    x = (torch.randperm(N * C * H * W).float() - 1000.0).view(N, C, H, W) / 7.0
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, (ph, pw), (sh, sw), (pad_h, pad_w))
    dy = torch.randn_like(yr)
    yr.backward(dy)
    y, idx = hip.maxpool_fwd(x.cuda().contiguous(memory_format=CL), ph, pw, sh, sw, pad_h, pad_w)
    assert y.dtype == torch.float32 and torch.equal(y.cpu(), yr.detach())
    dx = hip.maxpool_bwd(dy.cuda().contiguous(memory_format=CL), idx, (N, C, H, W), ph, pw, sh, sw, pad_h, pad_w)
    assert torch.equal(dx.cpu(), xr.grad)
