"""Streaming 1x1 conv kernel (csrc/kernels/g1s.hip) against a plain PyTorch fp32 reference and
against the gathered-GEMM path it replaces (gemm2.hip, g1s_enable(0)).

Forward (+ bias / residual / ReLU, + Welford BatchNorm statistics of the stored values) and the
stride-1 data gradient with the backward-BatchNorm fusion (ReLU mask + g / g*xhat sums) of the
producing layer, on ResNet-50 bottleneck shapes (K = 64 / 128 in VGPRs, 256 / 512 in LDS).
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
    assert h.kernels().arch == "gfx950"
    yield h
    h.kernels().g1s_enable(1)


FWD_CASES = [
    # N, Ci, H, W, Co, stride
    (4, 64, 16, 16, 256, 1),     # bottleneck expand (K = 64)
    (4, 64, 16, 16, 64, 1),      # layer-1 block-1 reduce (64 -> 64)
    (4, 128, 8, 8, 512, 1),      # layer-2 expand (K = 128)
    (8, 64, 8, 8, 128, 2),       # strided projection (ResNet-18 layer 2)
    (2, 128, 16, 16, 256, 2),    # strided projection, K = 128
    (64, 128, 4, 4, 128, 1),     # 4x4 maps: several images per 64-pixel tile
    (4, 256, 16, 16, 64, 1),     # layer-1 reduce (K = 256: weights in LDS)
    (2, 512, 8, 8, 128, 1),      # layer-2 reduce (K = 512)
    (4, 256, 16, 16, 128, 2),    # strided projection, K = 256
    (4, 32, 32, 32, 64, 1),      # K = 32 (ResNet-18 layer-1 projection)
    (4, 256, 4, 4, 64, 1),       # 2 tiles: trailing pixel ranges of a workgroup stay empty
]


@pytest.mark.parametrize("case", FWD_CASES)
def test_g1s_forward_stats(hip, case):
    N, Ci, H, W, Co, s = case
    K = hip.kernels()
    OH, OW = (H - 1) // s + 1, (W - 1) // s + 1
    assert K.g1s_rows(N * OH * OW, Co, Ci, 1) > 0
    torch.manual_seed(1)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, 1, 1) / math.sqrt(Ci)
    b = torch.randn(Co) + 2.0
    y_ref = F.conv2d(bf(x), bf(w), b, s, 0)
    xg = x.cuda().bfloat16().contiguous(memory_format=CL)
    wg = w.cuda().bfloat16().contiguous(memory_format=CL)
    outs = []
    for _ in range(2):
        y, partial = hip.conv2d_fwd(xg, wg, b.cuda(), (s, s), (0, 0), stats=True)
        assert partial[1] == K.g1s_rows(N * OH * OW, Co, Ci, 1)
        outs.append((y, hip.bn_stats(y, partial).clone()))
    (y, st), (y2, st2) = outs
    assert torch.equal(y, y2) and torch.equal(st, st2)  # deterministic
    assert rel_err(y, y_ref) < 1e-2, rel_err(y, y_ref)
    yd = y.double()
    assert rel_err(st[:Co], yd.mean((0, 2, 3))) < 1e-6
    var = yd.var((0, 2, 3), unbiased=False).cpu()
    assert ((st[Co:].double().cpu() - var).abs() / var).max() < 1e-3
    # same products in the same k order as the gathered GEMM: bit-identical outputs
    K.g1s_enable(0)
    try:
        y0, p0 = hip.conv2d_fwd(xg, wg, b.cuda(), (s, s), (0, 0), stats=True)
    finally:
        K.g1s_enable(1)
    assert torch.equal(y0, y)
    st0 = hip.bn_stats(y0, p0)
    assert rel_err(st, st0) < 1e-5


def test_g1s_forward_large_mean_stats(hip):
    """Welford rows about the wave's pivot: a 1e3 offset does not cancel the variance."""
    N, Ci, H, W, Co = 8, 64, 32, 32, 256
    torch.manual_seed(2)
    xg = torch.randn(N, Ci, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    wg = (torch.randn(Co, Ci, 1, 1) / math.sqrt(Ci)).cuda().bfloat16().contiguous(memory_format=CL)
    b = torch.full((Co,), 1e3, device="cuda")
    y, partial = hip.conv2d_fwd(xg, wg, b, (1, 1), (0, 0), stats=True)
    st = hip.bn_stats(y, partial)
    yd = y.double()
    var = yd.var((0, 2, 3), unbiased=False).cpu()
    assert rel_err(st[:Co], yd.mean((0, 2, 3))) < 1e-6
    assert ((st[Co:].double().cpu() - var).abs() / var).max() < 1e-3


@pytest.mark.parametrize("relu", [False, True])
def test_g1s_forward_residual_relu(hip, relu):
    N, Ci, H, W, Co = 4, 128, 8, 8, 256
    torch.manual_seed(3)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, 1, 1) / math.sqrt(Ci)
    b = torch.randn(Co)
    r = torch.randn(N, Co, H, W)
    ref = F.conv2d(bf(x), bf(w), b) + bf(r)
    if relu:
        ref = ref.clamp_min(0)
    y, _ = hip.conv2d_fwd(x.cuda().bfloat16().contiguous(memory_format=CL),
                          w.cuda().bfloat16().contiguous(memory_format=CL), b.cuda(), (1, 1), (0, 0),
                          residual=r.cuda().bfloat16().contiguous(memory_format=CL), relu=relu)
    assert rel_err(y, ref) < 1e-2, rel_err(y, ref)


DGRAD_CASES = [
    # N, C (dgrad output = the BN'd input channels), H, W, Co (dgrad K), relu, residual
    (4, 256, 16, 16, 64, True, False),   # layer-1 reduce conv's input gradient (K = 64, N = 256)
    (4, 512, 8, 8, 128, True, False),    # layer-2 reduce conv (K = 128)
    (4, 64, 16, 16, 64, False, False),   # BN without a ReLU
    (4, 256, 16, 16, 64, True, True),    # + the shortcut's gradient (block input)
    (4, 64, 16, 16, 256, True, False),   # expand conv's input gradient (K = 256)
    (2, 128, 8, 8, 512, True, True),     # K = 512 with residual
    # training-sized grids: several 32-pixel tiles per pixel range (statistics accumulated across
    # tiles in registers; the small cases above run one tile per range)
    (64, 256, 32, 32, 64, True, False),
    (64, 256, 32, 32, 256, True, False),
    (64, 512, 16, 16, 128, True, True),
]


@pytest.mark.parametrize("case", DGRAD_CASES)
def test_g1s_dgrad_bwd_bn_fusion(hip, case):
    """1x1 dgrad with the producing BatchNorm's ReLU mask + backward sums fused == dgrad then the
    standalone BN backward; and the unfused dgrad equals torch."""
    N, C, H, W, Co, relu, resid = case
    K = hip.kernels()
    assert K.g1s_rows(N * H * W, C, Co, 2) > 0
    torch.manual_seed(5)
    xb = (torch.randn(N, C, H, W) * 1.5 + 0.3).cuda().bfloat16().contiguous(memory_format=CL)
    g, bt = (torch.rand(C) + 0.5).cuda(), torch.randn(C).cuda()
    sums = hip.bn_stats(xb)
    mean, istd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    y = hip.bn_apply(xb, sums, N * H * W, g, bt, 1e-5, relu=relu, save=(mean, istd))
    yout = y if relu else None
    w = (torch.randn(Co, C, 1, 1) / math.sqrt(C)).cuda().bfloat16().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    dy = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    r = torch.randn(N, C, H, W).cuda().bfloat16().contiguous(memory_format=CL) if resid else None
    d_ref = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), residual=r)
    dx_t = torch.nn.grad.conv2d_input((N, C, H, W), w.float(), dy.float(), 1, 0)
    if resid:
        dx_t = dx_t + r.float()
    assert rel_err(d_ref, dx_t) < 1e-2
    dg0, db0 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx0, m0 = hip.bn_backward(d_ref, xb, yout, mean, istd, g, dg0, db0, want_masked=True)
    req = hip.BnbRequest("bn", yout, xb, mean, istd)
    d = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), residual=r, bnb=req)
    assert d._bnb[2] == K.g1s_rows(N * H * W, C, Co, 2)
    masked = d_ref.float() * (y.float() > 0) if relu else d_ref.float()
    assert rel_err(d, masked) < 1e-6
    dg1, db1 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx1, m1 = hip.bn_backward(d, xb, yout, mean, istd, g, dg1, db1, want_masked=True, fused=d._bnb[1:])
    assert rel_err(dx1, dx0) < 1e-2, rel_err(dx1, dx0)
    assert rel_err(dg1, dg0) < 1e-3, rel_err(dg1, dg0)
    assert rel_err(db1, db0) < 1e-3, rel_err(db1, db0)
    # deterministic
    d2 = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), residual=r, bnb=req)
    assert torch.equal(d, d2) and torch.equal(d._bnb[1], d2._bnb[1])


@pytest.mark.parametrize("case", [(32, 1024, 8, 8, 256), (32, 2048, 4, 4, 512), (8, 1024, 4, 4, 64)])
def test_hconv_1x1_k1024(hip, case, monkeypatch):
    """K >= 1024 1x1 convs on small grids (not on g1s) on the split-K halo
    kernel — forward with statistics and the data gradient, against torch fp32 and the gathered
    GEMM (the switch off)."""
    N, Ci, H, W, Co = case
    torch.manual_seed(7)
    x = torch.randn(N, Ci, H, W)
    w = torch.randn(Co, Ci, 1, 1) / math.sqrt(Ci)
    xg = x.cuda().bfloat16().contiguous(memory_format=CL)
    wg = w.cuda().bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(wg)
    outs = {}
    for on in (False, True):
        monkeypatch.setattr(fusion, "HCONV_1X1", on)
        y, partial = hip.conv2d_fwd(xg, wg, None, (1, 1), (0, 0), stats=True)
        st = hip.bn_stats(y, partial).clone()
        dx = hip.conv2d_dgrad(dy, wt, (N, Ci, H, W), (1, 1), (0, 0))
        torch.cuda.synchronize()
        outs[on] = (y, st, dx)
    y, st, dx = outs[True]
    y_ref = F.conv2d(bf(x), bf(w))
    assert rel_err(y, y_ref) < 1e-2
    assert rel_err(y, outs[False][0]) < 1e-2
    yd = y.double()
    assert rel_err(st[:Co], yd.mean((0, 2, 3))) < 1e-5
    var = yd.var((0, 2, 3), unbiased=False).cpu()
    assert ((st[Co:].double().cpu() - var).abs() / var).max() < 1e-3
    dx_t = torch.nn.grad.conv2d_input((N, Ci, H, W), wg.float(), dy.float(), 1, 0)
    assert rel_err(dx, dx_t) < 1e-2
    assert rel_err(dx, outs[False][2]) < 1e-2
