"""Every conv call of the C++ engine's production steps against an fp32 reference.

The C++ trainer (bin/tiny_imagenet_resnet18, the engine bench.py times) steps ResNet-18-tiny at
batch 64 and 256 and ResNet-50-tiny at batch 32 and 256 with ``DCNN_RECORD_OPS`` set: the GPU
backend (csrc/host/ops_gpu.hip) logs every conv it launches — direction (forward, data gradient,
weight gradient, RGB stem), the ConvShape, the epilogue options (bias, BatchNorm statistics,
residual, the pre-transposed dgrad operand, the fused BatchNorm backward with or without its ReLU
mask, the deferred split-K reduce) and the routing decision. Each distinct tuple is replayed once
through the same C++ entry points (the C ABI of csrc/host/capi.cpp on libdcnn.so, device pointers of
torch tensors: the C++ fusion plumbing, workspaces and split-K plans, not the Python wrappers) on
random data of exactly that geometry, and compared with PyTorch fp32 on the same bf16 inputs:

* outputs / data gradients: relative L2 < 1e-2, max error < 3e-2 of the reference's max;
* forward BatchNorm statistics: the epilogue's Welford rows, merged in float64, against the mean /
  variance of the kernel's own stored output;
* fused BatchNorm backward: the ReLU mask applied to dx, and the rows' (sum dx', sum dx' * xhat)
  against the same sums of the kernel's own output;
* weight / bias gradients (split-K slabs + the batched reduce): relative L2 < 5e-3.

A negative control injects a fault into the C++ dgrad plumbing (the BatchNorm ReLU mask operand
dropped, capi.cpp dcnn_c_set_fault) and requires the comparison to fail.
Reference parity: unit_tests/conv2d_layer_test.cpp:660-990, unit_tests/layer_device_agnosticity_test.cpp:60-103.
"""
import ctypes
import json
import os
import subprocess

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "dcnn_amd", "bin", "tiny_imagenet_resnet18")
LIB = os.path.join(ROOT, "dcnn_amd", "libdcnn.so")
CL = torch.channels_last
CONFIGS = [("resnet18_tiny_imagenet", 64), ("resnet18_tiny_imagenet", 256),
           ("resnet50_tiny_imagenet", 32), ("resnet50_tiny_imagenet", 256)]
P = ctypes.c_void_p


def _lib():
    L = ctypes.CDLL(LIB)
    L.dcnn_c_last_error.restype = ctypes.c_char_p
    for name in ("dcnn_c_conv_fwd", "dcnn_c_conv_dgrad", "dcnn_c_conv_wgrad", "dcnn_c_stem_fwd",
                 "dcnn_c_stem_wgrad", "dcnn_c_copy"):
        getattr(L, name).restype = ctypes.c_int
    return L


def _ok(L, rc):
    assert rc == 0, L.dcnn_c_last_error().decode()


_TUPLES = None


def _record(tmp_dir):
    out = []
    for name, b in CONFIGS:
        path = os.path.join(tmp_dir, f"{name}_{b}.jsonl")
        env = dict(os.environ, DCNN_RECORD_OPS=path)
        r = subprocess.run([EXE, "--device", "GPU", "--model", name, "--batch", str(b), "--steps", "1", "--warmup", "1",
                            "--bench", "--eager", "--loss", "softmax_ce"], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-3000:]
        with open(path) as f:
            out += [(json.loads(l), f"{name}@{b}") for l in f if l.strip()]
    return out


def _tuples(tmp_path_factory):
    """Distinct recorded conv tuples over the four configurations (first occurrence order)."""
    global _TUPLES
    if _TUPLES is None:
        seen = {}
        for c, where in _record(str(tmp_path_factory.mktemp("rec"))):
            seen.setdefault(json.dumps(c, sort_keys=True), (c, where))
        _TUPLES = list(seen.values())
    return _TUPLES


def _close(out, ref, what, rel=1e-2, mx=3e-2):
    out, ref = out.double(), ref.double()
    e = (out - ref).norm() / ref.norm().clamp_min(1e-30)
    m = (out - ref).abs().max() / ref.abs().max().clamp_min(1e-30)
    assert e < rel and m < mx, f"{what}: rel L2 {float(e):.3e}, max {float(m):.3e}"


def _bf(t):
    return t.to(torch.bfloat16)


def _slab(L, ptr, rows, width, C):
    t = torch.empty(rows, width, C, device="cuda")
    _ok(L, L.dcnn_c_copy(P(t.data_ptr()), P(ptr), ctypes.c_size_t(t.numel() * 4)))
    return t.double()


def _check_stats(L, y, ptr, rows):
    """Forward epilogue rows (count, mean, M2) merged in float64 == the stored output's moments."""
    C = y.shape[1]
    yd = y.double()
    s = _slab(L, ptr, rows, 3, C)
    n, mu, m2 = s[:, 0], s[:, 1], s[:, 2]
    tot = n.sum(0)
    mean = (n * mu).sum(0) / tot
    var = (m2.sum(0) + (n * (mu - mean) ** 2).sum(0)) / tot
    assert float(tot[0]) == y.numel() // C, "statistics rows: pixel count"
    rm, rv = yd.mean((0, 2, 3)), yd.var((0, 2, 3), unbiased=False)
    assert (mean - rm).abs().max() < 1e-4 * (1 + rm.abs().max()), "forward statistics: mean"
    assert ((var - rv).abs() / rv.clamp_min(1e-12)).max() < 1e-3, "forward statistics: variance"


def _replay(L, c, g):
    dev = "cuda"
    op = c["op"]
    sh = c["shape"]
    N, Ci, H, W, Co, KH, KW, SH, SW, PH, PW, OH, OW = sh
    shape = (ctypes.c_int * 13)(*sh)
    w = _bf(torch.randn(Co, Ci, KH, KW, generator=g) * (2.0 / (Ci * KH * KW)) ** 0.5).to(dev).contiguous(memory_format=CL)
    slab, rows = ctypes.c_void_p(), ctypes.c_int(0)
    torch.cuda.synchronize()
    if op in ("stem_fwd", "stem_wgrad"):
        x = torch.randn(N, Ci, H, W, generator=g).to(dev)
        if op == "stem_fwd":
            bias = torch.randn(Co, generator=g).to(dev) if c["bias"] else None
            y = torch.empty(N, Co, H, W, dtype=torch.bfloat16, device=dev).contiguous(memory_format=CL)
            _ok(L, L.dcnn_c_stem_fwd(P(x.data_ptr()), P(w.data_ptr()), P(bias.data_ptr() if bias is not None else 0),
                                     P(y.data_ptr()), shape, int(c["stats"]), ctypes.byref(slab), ctypes.byref(rows)))
            _close(y.float(), F.conv2d(x, w.float(), bias, 1, 1), "stem forward")
            if c["stats"]:
                _check_stats(L, y, slab.value, rows.value)
        else:
            dy = _bf(torch.randn(N, Co, H, W, generator=g)).to(dev).contiguous(memory_format=CL)
            gw = torch.zeros(Co, Ci, 3, 3, device=dev).contiguous(memory_format=CL)
            gb = torch.zeros(Co, device=dev) if c["bias"] else None
            _ok(L, L.dcnn_c_stem_wgrad(P(dy.data_ptr()), P(x.data_ptr()), P(gw.data_ptr()),
                                       P(gb.data_ptr() if gb is not None else 0), shape, int(c["deferred"])))
            _close(gw, torch.nn.grad.conv2d_weight(x, (Co, Ci, 3, 3), dy.float(), 1, 1), "stem weight gradient", rel=5e-3)
            if gb is not None:
                _close(gb, dy.float().sum((0, 2, 3)), "stem bias gradient", rel=1e-4, mx=1e-4)
        return
    x = _bf(torch.randn(N, Ci, H, W, generator=g)).to(dev).contiguous(memory_format=CL)
    if op == "fwd":
        bias = torch.randn(Co, generator=g).to(dev) if c["bias"] else None
        y = torch.empty(N, Co, OH, OW, dtype=torch.bfloat16, device=dev).contiguous(memory_format=CL)
        _ok(L, L.dcnn_c_conv_fwd(P(x.data_ptr()), P(w.data_ptr()), P(bias.data_ptr() if bias is not None else 0),
                                 P(y.data_ptr()), shape, int(c["stats"]), ctypes.byref(slab), ctypes.byref(rows)))
        _close(y.float(), F.conv2d(x.float(), w.float(), bias, (SH, SW), (PH, PW)), "forward")
        if c["stats"]:
            assert rows.value > 0, "the statistics epilogue was not honoured"
            _check_stats(L, y, slab.value, rows.value)
    elif op == "dgrad":
        dy = _bf(torch.randn(N, Co, OH, OW, generator=g)).to(dev).contiguous(memory_format=CL)
        res = _bf(torch.randn(N, Ci, H, W, generator=g)).to(dev).contiguous(memory_format=CL) if c["residual"] else None
        dx = torch.empty(N, Ci, H, W, dtype=torch.bfloat16, device=dev).contiguous(memory_format=CL)
        xb = yb = mean = istd = None
        if c["bnb"]:
            xb = _bf(torch.randn(N, Ci, H, W, generator=g) * 2 + 0.5).to(dev).contiguous(memory_format=CL)
            mean = xb.float().mean((0, 2, 3)).contiguous()
            istd = torch.rsqrt(xb.float().var((0, 2, 3), unbiased=False) + 1e-5).contiguous()
            if c["bnb_mask"]:
                gam = torch.randn(Ci, generator=g).to(dev)
                bet = torch.randn(Ci, generator=g).to(dev)
                yb = _bf(((xb.float() - mean[None, :, None, None]) * (istd * gam)[None, :, None, None]
                          + bet[None, :, None, None]).clamp_min(0)).contiguous(memory_format=CL)
        ptr = lambda t: P(t.data_ptr() if t is not None else 0)  # noqa: E731
        _ok(L, L.dcnn_c_conv_dgrad(ptr(dy), ptr(w), int(c["w_t"]), ptr(dx), shape, ptr(res), int(c["bnb"]), ptr(yb),
                                   ptr(xb), ptr(mean), ptr(istd), ctypes.byref(slab), ctypes.byref(rows)))
        ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w.float(), dy.float(), (SH, SW), (PH, PW))
        if res is not None:
            ref = ref + res.float()
        if yb is not None:
            ref = ref * (yb.float() > 0)
        _close(dx.float(), ref, "data gradient")
        if c["bnb"] and rows.value > 0:
            r = rows.value
            s = _slab(L, slab.value, r, 2, Ci).sum(0)
            d = dx.double()
            xhat = (xb.double() - mean.double()[None, :, None, None]) * istd.double()[None, :, None, None]
            ref_s = torch.stack([d.sum((0, 2, 3)), (d * xhat).sum((0, 2, 3))])
            scale = ref_s.abs().max(1, keepdim=True).values.clamp_min(1e-30)
            assert ((s - ref_s).abs() / scale).max() < 1e-4, "fused BatchNorm backward sums"
    else:  # wgrad
        dy = _bf(torch.randn(N, Co, OH, OW, generator=g)).to(dev).contiguous(memory_format=CL)
        gw = torch.zeros(Co, Ci, KH, KW, device=dev).contiguous(memory_format=CL)
        gb = torch.zeros(Co, device=dev) if c["bias"] else None
        _ok(L, L.dcnn_c_conv_wgrad(P(dy.data_ptr()), P(x.data_ptr()), P(gw.data_ptr()),
                                   P(gb.data_ptr() if gb is not None else 0), shape, int(c["deferred"])))
        ref = torch.nn.grad.conv2d_weight(x.float(), (Co, Ci, KH, KW), dy.float(), (SH, SW), (PH, PW))
        _close(gw, ref, "weight gradient", rel=5e-3)
        if gb is not None:
            _close(gb, dy.float().sum((0, 2, 3)), "bias gradient", rel=1e-4, mx=1e-4)


def test_cpp_recorded_tuples_cover_the_engine(tmp_path_factory):
    tups = _tuples(tmp_path_factory)
    ops = {c["op"] for c, _ in tups}
    assert {"fwd", "dgrad", "wgrad", "stem_fwd", "stem_wgrad"} <= ops, ops
    # the engine's fusions are exercised: statistics epilogues, the fused BN backward with and
    # without its mask, residual dgrads, pre-transposed operands, deferred split-K reduces
    assert any(c["op"] == "fwd" and c["stats"] for c, _ in tups)
    assert any(c["op"] == "dgrad" and c["bnb"] and c["bnb_mask"] for c, _ in tups)
    assert any(c["op"] == "dgrad" and c["w_t"] for c, _ in tups)
    assert any(c["op"] == "wgrad" and c["deferred"] for c, _ in tups)
    assert len({(c["op"], c["route"]) for c, _ in tups}) >= 6
    assert len(tups) >= 40, len(tups)


def test_cpp_every_recorded_tuple_matches_fp32(tmp_path_factory):
    L = _lib()
    g = torch.Generator().manual_seed(17)
    done = 0
    for c, where in _tuples(tmp_path_factory):
        try:
            _replay(L, c, g)
        except AssertionError as e:
            raise AssertionError(f"{where} {c}: {e}") from None
        done += 1
        torch.cuda.empty_cache()
    assert done == len(_tuples(tmp_path_factory))


def test_cpp_geometry_catches_a_broken_bnb_mask(tmp_path_factory):
    """Negative control: the dgrad epilogue without its ReLU mask must fail the comparison."""
    L = _lib()
    masked = [c for c, _ in _tuples(tmp_path_factory) if c["op"] == "dgrad" and c["bnb"] and c["bnb_mask"]]
    assert masked
    g = torch.Generator().manual_seed(5)
    L.dcnn_c_set_fault(1)
    try:
        with pytest.raises(AssertionError, match="data gradient|fused BatchNorm"):
            _replay(L, masked[0], g)
    finally:
        L.dcnn_c_set_fault(0)
    _replay(L, masked[0], torch.Generator().manual_seed(5))  # and passes again without the fault
