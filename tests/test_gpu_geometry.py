"""Every production conv geometry against an fp32 reference.

One eager training step of each BASELINE GPU model — ResNet-18-tiny at batch 64 and 256,
ResNet-50-tiny at batch 32 and 256 (the pipeline micro-batch and the single-GPU batch) — runs
under ``hip.record_convs()``, which logs every conv the step launches: direction (forward, data
gradient, weight gradient, RGB stem), shapes, stride / padding, the epilogue options (bias,
residual, ReLU, BatchNorm statistics, the fused BatchNorm backward with or without its ReLU mask)
and the routing table's decision (csrc/kernels/conv_route.cpp). Nothing is hand-picked: each
distinct recorded tuple is then replayed once on random data of exactly that geometry (so the
kernel variant, tile plan, split-K count and grid are the production ones — e.g. the K = 128 1x1
data gradient at ResNet-50 batch 256 with several tiles per pixel range, the case that computed
on stale operands before commit 070cf26) and compared with PyTorch fp32 on the same bf16 inputs:

* outputs: relative L2 error < 1e-2 and max error < 3e-2 of the reference's max (bf16 output
  rounding + fp32 accumulation order);
* forward BatchNorm statistics (the epilogue's Welford rows, reduced): mean / variance of the
  kernel's own stored output, in float64;
* fused BatchNorm backward (the dgrad epilogue): the ReLU mask applied to the data gradient and
  the sums (sum dy', sum dy' * xhat) of the kernel's own output;
* weight gradients (split-K slabs + the reduce): relative L2 error < 5e-3.

Reference parity: unit_tests/conv2d_layer_test.cpp:660-990 (ResNet layer shapes),
unit_tests/layer_device_agnosticity_test.cpp:60-103.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
CONFIGS = [("resnet18_tiny_imagenet", 64), ("resnet18_tiny_imagenet", 256),
           ("resnet50_tiny_imagenet", 32), ("resnet50_tiny_imagenet", 256)]


def _record(model_name, batch):
    from dcnn_amd.models import INPUT_SHAPES, NUM_CLASSES, create_model
    from dcnn_amd.nn import Adam, LossFactory
    from dcnn_amd.ops import hip
    from dcnn_amd.runtime.step import TrainStep
    m = create_model(model_name)
    m.set_seed(3)
    m.set_device("GPU:0")
    m.initialize()
    m.set_first_layer_input_grad(False)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(m, LossFactory.create("softmax_crossentropy"), opt, use_graph=False)
    C, H, W = INPUT_SHAPES[model_name]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(batch, C, H, W, generator=g).cuda()
    y = torch.randint(0, NUM_CLASSES[model_name], (batch,), generator=g).cuda()
    with hip.record_convs() as calls:
        st(x, y)
    torch.cuda.synchronize()
    return calls


_TUPLES = None


def _tuples():
    """Distinct recorded conv tuples over the four configurations (first occurrence order)."""
    global _TUPLES
    if _TUPLES is None:
        seen = {}
        for name, b in CONFIGS:
            for c in _record(name, b):
                key = tuple(sorted(c.items()))
                seen.setdefault(key, (c, f"{name}@{b}"))
        _TUPLES = list(seen.values())
    return _TUPLES


def _close(out, ref, what, rel=1e-2, mx=3e-2):
    out, ref = out.double(), ref.double()
    e = (out - ref).norm() / ref.norm().clamp_min(1e-30)
    m = (out - ref).abs().max() / ref.abs().max().clamp_min(1e-30)
    assert e < rel and m < mx, f"{what}: rel L2 {float(e):.3e}, max {float(m):.3e}"


def _bf(t):
    return t.to(torch.bfloat16)


def _replay(c, g):
    from dcnn_amd.ops import hip
    K = hip.kernels()
    dev = "cuda"
    op = c["op"]
    N, Ci, H, W = c["x"]
    Co, _, KH, KW = c["w"]
    w = _bf(torch.randn(Co, Ci, KH, KW, generator=g) * (2.0 / (Ci * KH * KW)) ** 0.5).to(dev)
    if op in ("stem_fwd", "stem_wgrad"):
        x = torch.randn(N, Ci, H, W, generator=g).to(dev)
        if op == "stem_fwd":
            bias = torch.randn(Co, generator=g).to(dev) if c["bias"] else None
            y, part = hip.stem_conv_fwd(x, w.float(), bias, stats=c["stats"])
            ref = F.conv2d(x, w.float(), bias, 1, 1)
            _close(y.float(), ref, "stem forward")
            if c["stats"]:
                _check_stats(hip, y, part)
        else:
            dy = _bf(torch.randn(N, Co, H, W, generator=g)).to(dev).contiguous(memory_format=CL)
            gw = torch.zeros(Co, Ci, 3, 3, device=dev)
            gb = torch.zeros(Co, device=dev) if c["bias"] else None
            hip.stem_conv_wgrad(dy, x, gw, gb)
            ref = torch.nn.grad.conv2d_weight(x, (Co, Ci, 3, 3), dy.float(), 1, 1)
            _close(gw, ref, "stem weight gradient", rel=5e-3)
            if gb is not None:
                _close(gb, dy.float().sum((0, 2, 3)), "stem bias gradient", rel=1e-4, mx=1e-4)
        torch.cuda.synchronize()
        return
    sh, sw = c["stride"]
    ph, pw = c["pad"]
    OH, OW = hip.conv_out_hw(H, W, KH, KW, sh, sw, ph, pw)
    x = _bf(torch.randn(N, Ci, H, W, generator=g)).to(dev).contiguous(memory_format=CL)
    if op == "fwd":
        bias = torch.randn(Co, generator=g).to(dev) if c["bias"] else None
        res = _bf(torch.randn(N, Co, OH, OW, generator=g)).to(dev).contiguous(memory_format=CL) if c["residual"] else None
        if c["padded_w"]:  # RGB conv: channels zero-padded to 8 (Conv2D.forward)
            xa = hip.to_act_padded(x, 8)
            wa = hip.pad_weight_channels(w.contiguous(memory_format=CL), 8)
        else:
            xa, wa = x, w.contiguous(memory_format=CL)
        y, part = hip.conv2d_fwd(xa, wa, bias, (sh, sw), (ph, pw), stats=c["stats"], residual=res, relu=c["relu"],
                                 out_fp32=c["out_fp32"])
        ref = F.conv2d(x.float(), w.float(), bias, (sh, sw), (ph, pw))
        if res is not None:
            ref = ref + res.float()
        if c["relu"]:
            ref = ref.clamp_min(0)
        _close(y.float(), ref, "forward")
        if c["stats"]:
            _check_stats(hip, y, part)
    elif op == "dgrad":
        dy = _bf(torch.randn(N, Co, OH, OW, generator=g)).to(dev).contiguous(memory_format=CL)
        wt = hip.conv_weight_t(w.contiguous(memory_format=CL))
        res = _bf(torch.randn(N, Ci, H, W, generator=g)).to(dev).contiguous(memory_format=CL) if c["residual"] else None
        req = None
        if c["bnb"]:
            xb = _bf(torch.randn(N, Ci, H, W, generator=g) * 2 + 0.5).to(dev).contiguous(memory_format=CL)
            mean = xb.float().mean((0, 2, 3))
            istd = torch.rsqrt(xb.float().var((0, 2, 3), unbiased=False) + 1e-5)
            yb = None
            if c["bnb_mask"]:
                gam = torch.randn(Ci, generator=g).to(dev)
                bet = torch.randn(Ci, generator=g).to(dev)
                yb = _bf(((xb.float() - mean[None, :, None, None]) * (istd * gam)[None, :, None, None]
                          + bet[None, :, None, None]).clamp_min(0)).contiguous(memory_format=CL)
            req = hip.BnbRequest(object(), yb, xb, mean.contiguous(), istd.contiguous())
        dx = hip.conv2d_dgrad(dy, wt, (N, Ci, H, W), (sh, sw), (ph, pw), residual=res, bnb=req)
        ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w.float(), dy.float(), (sh, sw), (ph, pw))
        if res is not None:
            ref = ref + res.float()
        if req is not None and req.y is not None:
            ref = ref * (req.y.float() > 0)
        _close(dx.float(), ref, "data gradient")
        if req is not None:
            assert getattr(dx, "_bnb", None) is not None, "the fused BatchNorm backward was not honoured"
            _, slab, rows, sums = dx._bnb
            s = hip.stat_reduce(1, slab, rows, Ci, sums).final().double().view(2, Ci)
            d = dx.double()
            xhat = (req.x.double() - req.mean.double()[None, :, None, None]) * req.istd.double()[None, :, None, None]
            ref_s = torch.stack([d.sum((0, 2, 3)), (d * xhat).sum((0, 2, 3))])
            scale = ref_s.abs().max(1, keepdim=True).values.clamp_min(1e-30)
            assert ((s - ref_s).abs() / scale).max() < 1e-4, "fused BatchNorm backward sums"
    else:  # wgrad
        dy = _bf(torch.randn(N, Co, OH, OW, generator=g)).to(dev).contiguous(memory_format=CL)
        xw = hip.to_act_padded(x, c["xpad"]) if c["xpad"] != Ci else x
        gw = torch.zeros(Co, Ci, KH, KW, device=dev).contiguous(memory_format=CL)
        gb = torch.zeros(Co, device=dev) if c["bias"] else None
        hip.conv2d_wgrad(dy, xw, (Co, Ci, KH, KW), (sh, sw), (ph, pw), gw, gb)
        ref = torch.nn.grad.conv2d_weight(x.float(), (Co, Ci, KH, KW), dy.float(), (sh, sw), (ph, pw))
        _close(gw, ref, "weight gradient", rel=5e-3)
        if gb is not None:
            _close(gb, dy.float().sum((0, 2, 3)), "bias gradient", rel=1e-4, mx=1e-4)
    torch.cuda.synchronize()


def _check_stats(hip, y, part):
    C = y.shape[1]
    s = hip.bn_stats(y, part).final().double().view(2, C)
    yd = y.double()
    mean = yd.mean((0, 2, 3))
    var = yd.var((0, 2, 3), unbiased=False)
    assert (s[0] - mean).abs().max() < 1e-4 * (1 + mean.abs().max()), "forward statistics: mean"
    assert ((s[1] - var).abs() / var.clamp_min(1e-12)).max() < 1e-3, "forward statistics: variance"


def test_recorded_conv_tuples_cover_the_routes():
    """The recording sees every routing decision family the four steps make."""
    from dcnn_amd.ops import hip
    K = hip.kernels()
    tups = _tuples()
    ops = {c["op"] for c, _ in tups}
    assert {"fwd", "dgrad", "wgrad", "stem_fwd", "stem_wgrad"} <= ops, ops
    routes = {(c["op"], c["route"]) for c, _ in tups}
    for r in (("fwd", K.ROUTE_HALO), ("fwd", K.ROUTE_G1S), ("fwd", K.ROUTE_GEMM_G2), ("dgrad", K.ROUTE_HALO),
              ("dgrad", K.ROUTE_G1S), ("dgrad", K.ROUTE_GEMM_G2), ("wgrad", K.ROUTE_HALO), ("wgrad", K.ROUTE_GEMM_G2),
              ("wgrad", K.ROUTE_HALO_S2)):
        assert r in routes, (r, sorted(routes))
    assert any(c["op"] == "dgrad" and c["bnb"] for c, _ in tups)
    assert any(c["op"] == "fwd" and c["stats"] for c, _ in tups)
    print(f"{len(tups)} distinct conv tuples")


def test_every_recorded_conv_tuple_matches_fp32_reference():
    tups = _tuples()
    g = torch.Generator().manual_seed(7)
    bad = []
    for c, where in tups:
        try:
            _replay(c, g)
        except AssertionError as e:
            bad.append(f"{where} {c}: {e}")
    print(f"replayed {len(tups)} tuples")
    assert not bad, "\n".join(bad)
