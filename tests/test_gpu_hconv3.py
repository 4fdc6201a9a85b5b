"""Third-generation halo conv (csrc/kernels/hconv3.hip): persistent, cross-tile pipelined; 64x64-per-wave
tiles, 3 taps per barrier, weights as the MFMA A operand (permuted rows: 16-byte epilogue stores). Checked against a plain PyTorch fp32 reference of
the same op and against the previous-generation kernel (hconv3_enable(0)) on every ResNet layer
geometry, with every epilogue option (bias, residual, ReLU, forward BN statistics, backward-BN
fusion) and split-K."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def hip():
    from dcnn_amd.ops import hip as H
    return H


# N, C (input channels), H, W, Co — the 16-wide-and-wider ResNet-18/50 layer geometries hconv3 runs
# (several 16x16 tiles per image, 64-channel tiles, split-K on the small grids)
CASES = [(4, 64, 32, 32, 64), (2, 64, 32, 64, 64), (4, 128, 16, 16, 128), (2, 64, 16, 16, 64),
         (4, 64, 16, 16, 128), (2, 256, 16, 16, 256), (64, 64, 32, 32, 64), (4, 512, 16, 16, 128),
         (4, 32, 32, 32, 64),  # 32 input channels: one chunk
         # small maps in the gutter layout: 2 x 2 images of 8 x 8 / 4 x 4 images of 4 x 4 per tile
         (4, 256, 8, 8, 256), (8, 128, 8, 8, 64), (64, 256, 8, 8, 256), (16, 512, 4, 4, 512),
         (32, 256, 4, 4, 128), (64, 512, 4, 4, 512)]


def _both(K, fn):
    """fn() on the hconv3 path and on the previous kernel."""
    out = []
    for on in (1, 0):
        K.hconv3_enable(on)
        try:
            out.append(fn())
        finally:
            K.hconv3_enable(1)
    return out


@pytest.mark.parametrize("case", CASES)
def test_hconv3_forward_epilogue(hip, case):
    K = hip.kernels()
    N, C, H, W, Co = case
    assert K.hconv_v3(N, H, W, C, Co, 9), case
    torch.manual_seed(31)
    x = torch.randn(N, C, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    b = torch.randn(Co).cuda() * 0.1 + 2.0   # large-ish mean: exercises the pivot-shifted statistics
    r = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)

    def run():
        y, part = hip.conv2d_fwd(x, w, b, (1, 1), (1, 1), stats=True, residual=r, relu=True)
        return y.clone(), hip.bn_stats(y, part).clone()

    (y3, s3), (y2, s2) = _both(K, run)
    y3b, s3b = run()
    assert torch.equal(y3, y3b) and torch.equal(s3, s3b)          # deterministic
    ref = F.relu(F.conv2d(x.float().cpu(), w.float().cpu(), b.cpu(), 1, 1) + r.float().cpu())
    assert rel_err(y3, ref) < 1e-2, rel_err(y3, ref)
    assert rel_err(y3, y2) < 5e-3
    # statistics of the stored output: fp64 reference
    yd = y3.double().cpu()
    assert rel_err(s3[:Co], yd.mean((0, 2, 3))) < 1e-5
    var = yd.var((0, 2, 3), unbiased=False)
    assert ((s3[Co:].double().cpu() - var).abs() / var).max() < 1e-3
    # plain conv (no epilogue options)
    y0 = hip.conv2d_fwd(x, w, None, (1, 1), (1, 1))[0]
    assert rel_err(y0, F.conv2d(x.float().cpu(), w.float().cpu(), None, 1, 1)) < 1e-2


@pytest.mark.parametrize("case", CASES)
def test_hconv3_dgrad(hip, case):
    K = hip.kernels()
    N, C, H, W, Co = case
    if not K.hconv_v3(N, H, W, Co, C, 9):
        pytest.skip("dgrad geometry not on hconv3")
    torch.manual_seed(32)
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    d3, d2 = _both(K, lambda: hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (1, 1)).clone())
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.float().cpu(), dy.float().cpu(), 1, 1)
    assert rel_err(d3, ref) < 1e-2
    assert rel_err(d3, d2) < 5e-3


@pytest.mark.parametrize("case", [(4, 64, 32, 32, 64), (4, 128, 16, 16, 128), (2, 256, 16, 16, 128)])
def test_hconv3_dgrad_bn_fusion(hip, case):
    """dgrad with the consuming BatchNorm's ReLU mask + backward statistics in the hconv3
    epilogue == the standalone BN backward of the unfused dgrad."""
    K = hip.kernels()
    N, C, H, W, Co = case
    assert K.hconv_v3(N, H, W, Co, C, 9)
    torch.manual_seed(33)
    xb = (torch.randn(N, C, H, W) * 1.5 + 0.3).cuda().bfloat16().contiguous(memory_format=CL)
    g, bt = (torch.rand(C) + 0.5).cuda(), torch.randn(C).cuda()
    sums = hip.bn_stats(xb)
    mean, istd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    y = hip.bn_apply(xb, sums, N * H * W, g, bt, 1e-5, relu=True, save=(mean, istd))
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    wt = hip.conv_weight_t(w)
    dy = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    d_ref = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (1, 1))
    dg0, db0 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx0, m0 = hip.bn_backward(d_ref, xb, y, mean, istd, g, dg0, db0, want_masked=True)
    req = hip.BnbRequest("bn", y, xb, mean, istd)
    d = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (1, 1), bnb=req)
    assert getattr(d, "_bnb", None) is not None
    assert rel_err(d, d_ref.float() * (y.float() > 0)) < 1e-6
    dg1, db1 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dx1, m1 = hip.bn_backward(d, xb, y, mean, istd, g, dg1, db1, want_masked=True, fused=d._bnb[1:])
    assert rel_err(dx1, dx0) < 1e-2
    assert rel_err(dg1, dg0) < 1e-3 and rel_err(db1, db0) < 1e-3
    assert rel_err(m1, m0) < 1e-6


def test_hconv3_small_maps_need_whole_image_groups(hip):
    """8 x 8 / 4 x 4 maps run as 2 x 2 / 4 x 4 image grids: a batch that does not fill the grid
    stays on the previous kernel."""
    K = hip.kernels()
    assert K.hconv_v3(8, 8, 8, 64, 64, 9) and not K.hconv_v3(6, 8, 8, 64, 64, 9)
    assert K.hconv_v3(16, 4, 4, 64, 64, 9) and not K.hconv_v3(8, 4, 4, 64, 64, 9)


def test_hconv3_split_k_matches_unsplit(hip):
    """A deep small grid: split-K (partials summed in split order by the tile's last workgroup) vs
    one workgroup per tile; repeated split launches bit-identical."""
    K = hip.kernels()
    N, C, H, W, Co = 4, 512, 16, 16, 128
    assert K.hconv_splits(N, H, W, C, Co, 9) > 1
    torch.manual_seed(34)
    x = torch.randn(N, C, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    b = torch.randn(Co).cuda()
    outs = []
    prev = K.hconv_split_target()
    try:
        for target in (512, 512, 0):
            K.hconv_set_split_target(target)
            y, part = hip.conv2d_fwd(x, w, b, (1, 1), (1, 1), stats=True, relu=True)
            outs.append((y.clone(), hip.bn_stats(y, part).clone()))
    finally:
        K.hconv_set_split_target(prev)
    (y1, s1), (y2, s2), (y0, s0) = outs
    assert torch.equal(y1, y2) and torch.equal(s1, s2)
    assert rel_err(y1, y0) < 5e-3 and rel_err(s1, s0) < 1e-3
    ref = F.relu(F.conv2d(x.float().cpu(), w.float().cpu(), b.cpu(), 1, 1))
    assert rel_err(y1, ref) < 1e-2


@pytest.fixture
def grid_cap(hip):
    K = hip.kernels()
    yield K
    K.hconv3_set_grid_cap(0)


@pytest.mark.parametrize("cap", [1, 3, 7])
@pytest.mark.parametrize("case", [(4, 64, 32, 32, 64), (4, 128, 16, 16, 128), (2, 256, 16, 16, 256),
                                  (4, 512, 16, 16, 128), (4, 32, 32, 32, 64), (16, 256, 8, 8, 256),
                                  (32, 512, 4, 4, 512)])
def test_hconv3_persistent_items_match(hip, grid_cap, case, cap):
    """Few workgroups walking many items (cross-item halo / weight prefetch, the next item's W(0,1)
    issued before the epilogue stores, split-K items in the stream): bit-identical to one item per
    workgroup, for the forward with every epilogue option and the dgrad with the BN fusion."""
    K = grid_cap
    N, C, H, W, Co = case
    torch.manual_seed(35)
    x = torch.randn(N, C, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(Co, C, 3, 3) / math.sqrt(9 * C)).cuda().bfloat16().contiguous(memory_format=CL)
    b = torch.randn(Co).cuda() * 0.1 + 1.0
    r = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)

    def fwd():
        y, part = hip.conv2d_fwd(x, w, b, (1, 1), (1, 1), stats=True, residual=r, relu=True)
        y1, part1 = hip.conv2d_fwd(x, w, None, (1, 1), (1, 1), stats=True)  # EPI=1 instance
        return y.clone(), hip.bn_stats(y, part).clone(), y1.clone(), hip.bn_stats(y1, part1).clone()

    K.hconv3_set_grid_cap(0)
    ref = fwd()
    K.hconv3_set_grid_cap(cap)
    got = fwd()
    for a_, b_ in zip(got, ref):
        assert torch.equal(a_, b_)
    if not K.hconv_v3(N, H, W, Co, C, 9) or C % 64:
        return
    # dgrad + backward-BN fusion (EPI=2 instance)
    xb = (torch.randn(N, C, H, W) * 1.5 + 0.3).cuda().bfloat16().contiguous(memory_format=CL)
    sums = hip.bn_stats(xb)
    mean, istd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    g_, bt = (torch.rand(C) + 0.5).cuda(), torch.randn(C).cuda()
    y = hip.bn_apply(xb, sums, N * H * W, g_, bt, 1e-5, relu=True, save=(mean, istd))
    wt = hip.conv_weight_t(w)
    dy = torch.randn(N, Co, H, W).cuda().bfloat16().contiguous(memory_format=CL)
    req = hip.BnbRequest("bn", y, xb, mean, istd)

    def dgrad():
        d = hip.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (1, 1), bnb=req)
        return d.clone(), d._bnb[1].clone()

    K.hconv3_set_grid_cap(0)
    d0, s0 = dgrad()
    K.hconv3_set_grid_cap(cap)
    d1, s1 = dgrad()
    assert torch.equal(d0, d1) and torch.equal(s0, s1)
