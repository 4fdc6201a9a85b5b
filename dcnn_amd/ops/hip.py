"""Torch-tensor front end of the HIP/CDNA4 kernel library (GPU path of every layer).

Activations are NHWC in memory (torch ``channels_last``) so the channel dimension is the
contiguous GEMM-K dimension of the implicit-GEMM convolution; the logical shape stays NCHW
(the reference API/checkpoint layout). Conv weights are ``channels_last`` too, i.e. physical
``[Cout][KH][KW][Cin]`` — the K-contiguous B operand of the MFMA GEMM. All launches go to
PyTorch's current HIP stream; activations, statistics slabs and workspaces come from the native
per-step activation arena while a training step runs (runtime/arena.py; PyTorch's caching
allocator otherwise), so a whole training step can be captured into a hipGraph.
"""
from __future__ import annotations

import functools
import os

import torch

from . import fusion
from ._ext import dt_code, kernels, ptr, stream_ptr
from .hip_base import *  # noqa: F401,F403  (shared plumbing, re-exported)
from .hip_base import (BF16, CL, CONV_DGRAD, CONV_FWD, F32, PLAIN, _NOBNB, _check_act, _empty, _empty_like,
                       _g2_ok, _nbytes, _rc, _rec, _reduce_wb, _ticket, conv_out_hw)
from .hip_convx import *  # noqa: F401,F403
from .hip_convx import (conv2d_dgrad_im2col, conv2d_fwd_im2col, conv2d_wgrad_im2col, _im2col_ok,
                        stem_ok, stem_conv_fwd)
from .hip_layers import *  # noqa: F401,F403
from .hip_layers import zero_
from .hip_norm import *  # noqa: F401,F403


@functools.lru_cache(maxsize=1024)
def _fwd_taps(C, W, KH, KW, ph, pw):
    """Tap list of a forward conv: (dy, dx, src element offset, B-row element offset). Cached per
    geometry (eager launches rebuild no Python lists); the tuple is never mutated."""
    taps = []
    for ky in range(KH):
        for kx in range(KW):
            dy, dx = ky - ph, kx - pw
            taps.append((dy, dx, (dy * W + dx) * C, (ky * KW + kx) * C))
    return tuple(taps)



# ---- split-precision fp32 convolutions on the bf16 halo kernels
# An fp32 operand x is split once into bf16 hi = bf16(x), lo = bf16(x - hi). A conv sums over
# input channels, so concatenating channels computes the three significant partial products in
# ONE bf16 MFMA conv with fp32 accumulation:  X3 = [xh | xl | xh], W3 = [wh | wh | wl] (per tap)
# gives sum xh*wh + xl*wh + xh*wl = x*w up to the dropped xl*wl (~2^-16 relative). The fp32 3x3
# stride-1 convs (forward and dgrad) therefore run on hconv (3x the channels, fp32 epilogue), and
# their weight gradients on hwgrad with three (dY, X) channel windows of the same split rows:
# (dyh, xh), (dyh, xl), (dyl, xh). Other fp32 convs keep the exact f32-MFMA gathered GEMMs.
_F32_CONCAT = True


def set_f32_concat(on: bool) -> None:
    """Route eligible fp32 convs through the split-precision halo kernels (True) or the exact
    f32-MFMA gathered GEMMs (False)."""
    global _F32_CONCAT
    _F32_CONCAT = bool(on)


def get_f32_concat() -> bool:
    return _F32_CONCAT


def split3_rows(t, rows, C, pattern, out=None):
    """fp32 [rows][C] (dense) -> bf16 [rows][3C]: pattern 0 [hi|lo|hi], 1 [hi|hi|lo]."""
    if out is None:
        out = _empty((rows, 3 * C), BF16, t.device)
    kernels().split3_bf16(t.data_ptr(), out.data_ptr(), rows, C, pattern, stream_ptr())
    return out


def act_split3(t):
    """[xh | xl | xh] channel concatenation of an fp32 NHWC activation (N, 3C, H, W) channels_last
    bf16; cached on the tensor (a conv's forward split serves its weight gradient too)."""
    s = getattr(t, "_s3", None)
    if s is None:
        N, C, H, W = t.shape
        assert t.dtype == F32 and t.is_contiguous(memory_format=CL)
        s = _empty((N, 3 * C, H, W), BF16, t.device, True)
        split3_rows(t, N * H * W, C, 0, out=s)
        t._s3 = s
    return s


def _f32_concat_ok(C, Co):
    return _F32_CONCAT and C % 64 == 0 and Co % 64 == 0




# K >= 1024 1x1 convs on small grids run on the split-K halo kernel. Always on; tests flip it
# (monkeypatch) to compare the halo route against the gathered-GEMM route on the same shapes.


def _hconv_ok(N, OH, OW, H, W, sh, sw, Cs, Co, taps, wop, split3=False):
    """Halo-tiled direct conv applies to stride-1 'same' convs with a 1-pixel reach (3x3/pad 1
    forward and its dgrad) on 64-multiple channel counts. ``split3``: the caller is a 3 x bf16
    fp32 concat path (Cs = 3 x the real channels): 1x1 convs stay on the exact fp32 GEMM there."""
    if (sh, sw) != (1, 1) or (OH, OW) != (H, W) or len(taps) > 9:
        return False
    if any(abs(t[0]) > 1 or abs(t[1]) > 1 for t in taps):
        return False
    if len(taps) == 1 and not (fusion.HCONV_1X1 and not split3 and Cs >= 1024 and (N * OH * OW // 64) * (Co // 64) < 256):
        # 1x1: the plain GEMM is already read-once. Except K >= 1024 1x1 convs (not on the
        # streaming kernel) whose GEMM grid would be < 256 tiles: the halo kernel splits their K
        # over the channel chunks (ResNet-50 b32: 7.87k -> 7.92k img/s)
        return False
    return bool(kernels().hconv_supported(N, H, W, Cs, Co, len(taps)))


class _SplitWs:
    """Workspace of one split-K halo conv launch: kept referenced until the launch is enqueued
    (stream-ordered caching allocator: later reuse of the block is ordered after the kernel)."""
    keep = None


# split-precision fp32 convs never split: their error budget (~2^-16 per conv) is validated on
# the unsplit accumulation order, and an ill-conditioned batch-8 BatchNorm backward chain
# (tests/test_gpu_model.py::test_fp32_gpu_model_matches_cpu) amplifies any order change ~300x
_NOSPLIT = (1, 0, 0)
# exact fp32 3x3 stride-1 convs and data gradients on the persistent halo conv's fp32 instances
# (DCNN_H3_F32=0: the gathered f32 GEMM); launches counted for the tests
_H3_F32 = os.environ.get("DCNN_H3_F32", "1") == "1"
# and their weight gradients on the halo wgrad's fp32 instances (DCNN_HW_F32=0: gemm_t2f)
_HW_F32 = os.environ.get("DCNN_HW_F32", "1") == "1"
_H3_F32_STATS = {"fwd": 0, "dgrad": 0, "dgrad_bnb": 0, "wgrad": 0}


def _hconv_split(K, NB, H, W, Cs, N, ntaps, device):
    """(splits, partials pointer, ticket words pointer) for :func:`hconv` (hconv.hip split-K:
    small grids are split over 64-channel chunks, the last workgroup of a tile sums the partials
    in split order and runs the epilogue)."""
    s = K.hconv_splits(NB, H, W, Cs, N, ntaps)
    if s == 1:
        return 1, 0, 0
    tiles = K.hconv_tiles(NB, H, W, Cs, N, ntaps)
    part = _empty((tiles * s * K.hconv_tile_elems(NB, H, W, Cs, N, ntaps),), F32, device)
    _SplitWs.keep = part
    return s, part.data_ptr(), _ticket(device, tiles * 64, "hconv").data_ptr()




def conv2d_fwd(x, w, bias, stride, pad, *, stats=False, residual=None, relu=False, out_fp32=False):
    """y = conv(x, w) + bias  [+ residual] [ReLU]; optional BN partial statistics slab.

    x: (N,Ci,H,W) bf16 channels_last; w: (Co,Ci,KH,KW) bf16 channels_last (or a padded
    [Co][KH][KW][Cp] operand when Ci was padded to Cp, see ``pad_input_channels``).
    Returns (y, (slab, rows) | None).
    """
    _check_act(x, "conv2d_fwd.x")
    if (_CONV_ALGO == "im2col" and not out_fp32 and w.dim() == 4 and w.shape[1] == x.shape[1]
            and _im2col_ok(x.shape[1], w.shape[0])):
        return conv2d_fwd_im2col(x, w, bias, stride, pad, stats=stats, residual=residual, relu=relu)
    K = kernels()
    N, Ci, H, W = x.shape
    if w.dim() == 4 and w.shape[1] == Ci:
        Co, _, KH, KW = w.shape
        assert w.is_contiguous(memory_format=CL)
    else:  # padded operand [Co][KH][KW][Ci]
        Co, KH, KW, Cp = w.shape
        assert Cp == Ci and w.is_contiguous()
    assert x.dtype == w.dtype and x.dtype in (BF16, F32)
    sh, sw = stride
    ph, pw = pad
    OH, OW = conv_out_hw(H, W, KH, KW, sh, sw, ph, pw)
    M = N * OH * OW
    if residual is not None:
        assert tuple(residual.shape) == (N, Co, OH, OW) and residual.is_contiguous(memory_format=CL)
    if x.dtype == F32 and _f32_concat_ok(Ci, Co) and _hconv_ok(N, OH, OW, H, W, sh, sw, 3 * Ci, Co,
                                                                 _fwd_taps(3 * Ci, W, KH, KW, ph, pw), w, True):
        # split-precision fp32 on the bf16 halo conv (see _F32_CONCAT)
        xs = act_split3(x)
        ws = split3_rows(w, Co * KH * KW, Ci, 1)
        y = _empty((N, Co, OH, OW), F32, x.device, True)
        slab, rows, sums = None, 0, None
        if stats:
            rows = K.hconv_stat_rows(N, H, W, 3 * Ci, Co, KH * KW, 1)
            slab = _empty((rows, 3, Co), F32, x.device)
            sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
        K.hconv(xs.data_ptr(), ws.data_ptr(), 0, _nbytes(xs), _nbytes(ws), N, H, W, 3 * Ci, Co, KH * KW * 3 * Ci,
                [(t[0], t[1], t[3]) for t in _fwd_taps(3 * Ci, W, KH, KW, ph, pw)], ptr(bias), 0, ptr(slab),
                int(relu), ptr(sums), 2 * Co if stats else 0, _NOBNB, y.data_ptr(), ptr(residual),
                *_NOSPLIT, stream_ptr())
        return y, ((slab, rows, sums) if stats else None)
    if (x.dtype == F32 and _H3_F32 and (KH, KW, sh, sw, ph, pw) == (3, 3, 1, 1, 1, 1) and w.dim() == 4
            and w.shape[1] == Ci):
        # exact fp32 3x3 on the persistent halo conv (hconv3 F32 instances: v_mfma_f32_16x16x4_f32)
        taps = [(t[0], t[1], t[3]) for t in _fwd_taps(Ci, W, KH, KW, ph, pw)]
        if len(taps) == 9 and K.hconv3_f32_splits(N, H, W, Ci, Co, 9):
            y = _empty((N, Co, OH, OW), F32, x.device, True)
            rows = K.hconv_stat_rows(N, H, W, 2 * Ci, Co, 9, 0) if stats else 0
            slab = _empty((rows, 3, Co), F32, x.device) if stats else None
            sums = _empty((2 * Co,), F32, x.device) if stats else None  # zeroed in-kernel
            if K.hconv3_f32(x.data_ptr(), w.data_ptr(), _nbytes(x), _nbytes(w), N, H, W, Ci, Co, KH * KW * Ci, taps,
                            ptr(bias), ptr(slab), int(relu), ptr(sums), 2 * Co if stats else 0, y.data_ptr(),
                            ptr(residual), *_hconv_split(K, N, H, W, 2 * Ci, Co, 9, x.device), stream_ptr()):
                _H3_F32_STATS["fwd"] += 1
                return y, ((slab, rows, sums) if stats else None)
    if x.dtype == F32:  # fp32 compute path: MFMA f32 16x16x4 gathered GEMM
        y = _empty((N, Co, OH, OW), F32, x.device, True)
        slab, rows, sums = None, 0, None
        if stats:
            rows = K.gemm_g2f_stat_rows(M, Co)
            slab = _empty((rows, 3, Co), F32, x.device)
            sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
        K.gemm_g2f(x.data_ptr(), w.data_ptr(), y.data_ptr(), _nbytes(x), _nbytes(w), M, Co, Ci, H, W, OH, OW, sh, sw,
                   _fwd_taps(Ci, W, KH, KW, ph, pw), KH * KW * Ci, Co, OH, OW, 1, 1, 0, 0, ptr(bias), ptr(residual),
                   ptr(slab), int(relu), ptr(sums), 2 * Co if stats else 0, _NOBNB, stream_ptr())
        return y, ((slab, rows, sums) if stats else None)
    # the shared routing table (csrc/kernels/conv_route.cpp, also used by the C++ host API)
    g1s_mode = (1 if stats else 0) if (w.dim() == 4 and (not stats or (residual is None and not relu))) else -1
    route = (K.conv_fwd_route(N, Ci, H, W, Co, KH, KW, sh, sw, ph, pw, OH, OW, g1s_mode)
             if not out_fp32 else K.ROUTE_GENERIC)
    if route == K.ROUTE_HALO and KH * KW == 1 and not fusion.HCONV_1X1:
        route = K.ROUTE_GEMM_G2
    _rec("fwd", x=tuple(x.shape), w=(Co, Ci, KH, KW), padded_w=not (w.dim() == 4 and w.shape[1] == Ci), stride=(sh, sw),
         pad=(ph, pw), stats=bool(stats), bias=bias is not None, residual=residual is not None, relu=bool(relu),
         route=int(route), out_fp32=bool(out_fp32))
    if route == K.ROUTE_G1S:
        # streaming 1x1 conv (g1s.hip): weights in registers, one statistics row per pixel range
        rows = K.g1s_rows(M, Co, Ci, 1 if stats else 0)
        if rows:
            y = _empty((N, Co, OH, OW), BF16, x.device, True)
            slab = _empty((rows, 3, Co), F32, x.device) if stats else None
            sums = _empty((2 * Co,), F32, x.device) if stats else None  # zeroed in-kernel
            K.g1s(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, Co, Ci, H, W, OH, OW, sh, ptr(bias), ptr(residual),
                  ptr(slab), int(relu), ptr(sums), 2 * Co if stats else 0, _NOBNB, 1 if stats else 0, stream_ptr())
            return y, ((slab, rows, sums) if stats else None)
    taps = _fwd_taps(Ci, W, KH, KW, ph, pw)
    if route == K.ROUTE_HALO and len(taps) == KH * KW:
        y = _empty((N, Co, OH, OW), BF16, x.device, True)
        slab, rows, sums = None, 0, None
        if stats:
            rows = K.hconv_stat_rows(N, H, W, Ci, Co, len(taps), 0)
            slab = _empty((rows, 3, Co), F32, x.device)
            sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
        K.hconv(x.data_ptr(), w.data_ptr(), y.data_ptr(), _nbytes(x), _nbytes(w), N, H, W, Ci, Co, KH * KW * Ci,
                [(t[0], t[1], t[3]) for t in taps], ptr(bias), ptr(residual), ptr(slab), int(relu), ptr(sums),
                2 * Co if stats else 0, _NOBNB, 0, 0, *_hconv_split(K, N, H, W, Ci, Co, KH * KW, x.device),
                stream_ptr())
        return y, ((slab, rows, sums) if stats else None)
    if route in (K.ROUTE_GEMM_G2, K.ROUTE_HALO, K.ROUTE_G1S):
        y = _empty((N, Co, OH, OW), BF16, x.device, True)
        slab, rows, sums = None, 0, None
        if stats:
            rows = K.gemm_g2_stat_rows(M, Co)
            slab = _empty((rows, 3, Co), F32, x.device)
            sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
        K.gemm_g2_grouped(x.data_ptr(), w.data_ptr(), y.data_ptr(), _nbytes(x), _nbytes(w), M, Co, Ci, H, W, OH, OW,
                          sh, sw, _fwd_taps(Ci, W, KH, KW, ph, pw), KH * KW * Ci, Co, OH, OW, 1, 1, 0, 0, ptr(bias),
                          ptr(residual), ptr(slab), int(relu), ptr(sums), 2 * Co if stats else 0, _NOBNB,
                          stream_ptr(), [])
        return y, ((slab, rows, sums) if stats else None)
    # generic fallback (odd channel counts): v1 kernels
    y = _empty((N, Co, OH, OW), F32 if out_fp32 else BF16, x.device, True)
    slab, rows = None, 0
    if stats:
        rows = K.gemm_nt_stat_rows(M, Co)
        slab = _empty((rows, 3, Co), F32, x.device)
    K.gemm_nt(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, Co, KH * KW * Ci, 0, KH * KW * Ci, Co, CONV_FWD,
              N, H, W, Ci, OH, OW, KH, KW, sh, sw, ph, pw, ptr(bias), ptr(residual), ptr(slab),
              int(out_fp32), int(relu), stream_ptr())
    sums = _empty((2 * Co,), F32, x.device) if stats else None
    return y, ((slab, rows, sums) if stats else None)


# ---- conv algorithm: implicit GEMM / halo kernels (default) or explicit im2col + GEMM
# (im2col.hip: the reference's lowering, src/nn/layers_impl/cuda/conv2d_ops.cu:78-98). Both run
# on the same MFMA GEMMs; im2col materialises the [N*OH*OW][KH*KW*C] column matrix in HBM.
_CONV_ALGO = os.environ.get("DCNN_CONV_ALGO", "implicit")
if _CONV_ALGO not in ("implicit", "im2col"):
    raise ValueError(f"DCNN_CONV_ALGO={_CONV_ALGO!r}: expected 'implicit' or 'im2col'")


def set_conv_algo(name: str) -> None:
    """Select the GPU convolution algorithm: ``"implicit"`` (implicit-GEMM / halo kernels) or
    ``"im2col"`` (explicit column matrix + plain GEMM)."""
    global _CONV_ALGO
    if name not in ("implicit", "im2col"):
        raise ValueError(f"unknown conv algorithm {name!r}")
    _CONV_ALGO = name


def get_conv_algo() -> str:
    return _CONV_ALGO



@functools.lru_cache(maxsize=1024)
def _dgrad_classes(H, W, OW, Co, KH, KW, sh, sw, ph, pw):
    """Stride-phase decomposition of a dgrad: ((ry, rx, GH, GW, taps) with taps, ...) and the
    phases no tap reaches; taps = (dy offset, dx offset, dy element offset, B-row offset).
    Cached per geometry (tuples, never mutated)."""
    classes, empty = [], []
    for ry in range(sh):
        for rx in range(sw):
            GH, GW = (H - ry + sh - 1) // sh, (W - rx + sw - 1) // sw
            if GH <= 0 or GW <= 0:
                continue
            taps = []
            for ky in range(KH):
                if (ry + ph - ky) % sh:
                    continue
                dyo = (ry + ph - ky) // sh
                for kx in range(KW):
                    if (rx + pw - kx) % sw:
                        continue
                    dxo = (rx + pw - kx) // sw
                    taps.append((dyo, dxo, (dyo * OW + dxo) * Co, (ky * KW + kx) * Co))
            (classes if taps else empty).append((ry, rx, GH, GW, tuple(taps)))
    return tuple(classes), tuple(empty)


def conv2d_dgrad(dy, wt, x_shape, stride, pad, *, residual=None, bnb=None):
    """dx = conv_transpose(dy, w) [+ residual];  wt = conv_weight_t(w).

    Strided convs are phase-decomposed: input pixels are split into stride^2 parity classes,
    each a dense GEMM over only the kernel taps that reach it (no MFMA work on zero taps).
    ``bnb`` (a :class:`BnbRequest`): fuse the consuming BatchNorm's ReLU mask and backward
    statistics into the epilogue (honoured on the bf16 MFMA paths; see ``dx._bnb``).
    """
    _check_act(dy, "conv2d_dgrad.dy")
    if _CONV_ALGO == "im2col" and _im2col_ok(x_shape[1], dy.shape[1]):
        return conv2d_dgrad_im2col(dy, wt, x_shape, stride, pad, residual=residual)
    K = kernels()
    N, Ci, H, W = x_shape
    Co, OH, OW = dy.shape[1], dy.shape[2], dy.shape[3]
    Ci2, KH, KW, Co2 = wt.shape
    assert Ci == Ci2 and Co == Co2
    if residual is not None:
        assert tuple(residual.shape) == (N, Ci, H, W) and residual.is_contiguous(memory_format=CL)
    sh, sw = stride
    ph, pw = pad
    f32 = dy.dtype == F32
    if f32:
        assert wt.dtype == F32, "fp32 dgrad needs an fp32 transposed weight (conv_weight_t(..., dtype=F32))"
    fuse_req = bnb is not None and fusion.BNB and not bnb.pooled and not f32 and bnb.x.dtype == BF16 \
        and tuple(bnb.x.shape) == (N, Ci, H, W)
    # the shared routing table (csrc/kernels/conv_route.cpp, also used by the C++ host API)
    route = K.conv_dgrad_route(N, Ci, H, W, Co, KH, KW, sh, sw, ph, pw, OH, OW, 2 if fuse_req else 0) \
        if not f32 else K.ROUTE_GEMM_G2
    if route == K.ROUTE_HALO and KH * KW == 1 and not fusion.HCONV_1X1:
        route = K.ROUTE_GEMM_G2
    if not f32:
        _rec("dgrad", x=tuple(x_shape), w=(Co, Ci, KH, KW), stride=(sh, sw), pad=(ph, pw),
             residual=residual is not None, bnb=bool(fuse_req), bnb_mask=bool(fuse_req and bnb.y is not None),
             route=int(route))
    if not f32 and route == K.ROUTE_GENERIC:
        dx = _empty((N, Ci, H, W), BF16, dy.device, True)
        Kd = KH * KW * Co
        K.gemm_nt(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N * H * W, Ci, Kd, 0, Kd, Ci, CONV_DGRAD,
                  N, OH, OW, Co, H, W, KH, KW, sh, sw, ph, pw, 0, ptr(residual), 0, 0, 0, stream_ptr())
        return dx
    classes, empty = _dgrad_classes(H, W, OW, Co, KH, KW, sh, sw, ph, pw)
    empty_class = bool(empty)
    odt = F32 if f32 else BF16
    allc = classes + empty
    if (not f32 and empty_class and len(classes) > 1 and fusion.G2_GROUP and len(allc) <= 4
            and len({(c[2], c[3]) for c in allc}) == 1 and (N * allc[0][2] * allc[0][3]) % 128 == 0):
        # phases no tap reaches join the grouped launch as zero-tap classes: their epilogue writes
        # the residual (or zeros), so there is no separate fill / copy pass. (With a single tap
        # class — 1x1 stride 2 — a zero fill + one class launch is faster: measured 1x1 s2 dgrads
        # 18 / 20 / 30 us grouped vs 18 / 16 / 22 us filled on the ResNet-18 layers.)
        GH, GW = allc[0][2], allc[0][3]
        M = len(allc) * N * GH * GW
        taps_all, groups = [], []
        for ry, rx, _, _, taps in allc:
            groups.append((len(taps_all), len(taps), ry, rx))
            taps_all += taps
        dx = _empty((N, Ci, H, W), BF16, dy.device, True)
        K.gemm_g2_grouped(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _nbytes(dy), _nbytes(wt), M, Ci, Co, OH, OW,
                          GH, GW, 1, 1, taps_all, KH * KW * Co, Ci, H, W, sh, sw, 0, 0, 0, ptr(residual), 0, 0, 0, 0,
                          _NOBNB, stream_ptr(), groups)
        return dx
    if empty_class:
        # positions no tap reaches keep the residual (or zero); a memset / async copy node, not a kernel
        dx = _empty((N, Ci, H, W), odt, dy.device, True)
        if residual is not None:
            dx.copy_(residual)
        else:
            zero_(dx)
    else:
        dx = _empty((N, Ci, H, W), odt, dy.device, True)
    st = stream_ptr()
    if (f32 and len(classes) == 1 and not empty_class and _f32_concat_ok(Co, Ci)
            and _hconv_ok(N, H, W, OH, OW, sh, sw, 3 * Co, Ci, classes[0][4], wt, True)):
        # split-precision fp32 dgrad on the bf16 halo conv (see _F32_CONCAT)
        dys = act_split3(dy)
        wts = split3_rows(wt, Ci * KH * KW, Co, 1)
        K.hconv(dys.data_ptr(), wts.data_ptr(), 0, _nbytes(dys), _nbytes(wts), N, OH, OW, 3 * Co, Ci,
                KH * KW * 3 * Co, [(t[0], t[1], 3 * t[3]) for t in classes[0][4]], 0, 0, 0, 0, 0, 0, _NOBNB,
                dx.data_ptr(), ptr(residual), *_NOSPLIT, st)
        return dx
    if (f32 and _H3_F32 and len(classes) == 1 and not empty_class and (KH, KW, sh, sw, ph, pw) == (3, 3, 1, 1, 1, 1)
            and len(classes[0][4]) == 9 and K.hconv3_f32_splits(N, OH, OW, Co, Ci, 9)):
        # exact fp32 data gradient on the persistent halo conv (transposed weights, reversed taps),
        # with the consuming BatchNorm's ReLU mask + backward statistics in the epilogue when asked
        fuse32 = (bnb is not None and fusion.BNB and not bnb.pooled and bnb.x.dtype == F32
                  and tuple(bnb.x.shape) == (N, Ci, H, W) and (bnb.y is None or bnb.y.dtype == F32))
        rows = K.hconv_stat_rows(N, H, W, 2 * Co, Ci, 9, 0) if fuse32 else 0
        slab = _empty((rows, 2, Ci), F32, dy.device) if fuse32 else None
        sums = _empty((2 * Ci,), F32, dy.device) if fuse32 else None  # zeroed in-kernel
        if K.hconv3_f32(dy.data_ptr(), wt.data_ptr(), _nbytes(dy), _nbytes(wt), N, OH, OW, Co, Ci, KH * KW * Co,
                        [(t[0], t[1], t[3]) for t in classes[0][4]], 0, ptr(slab), 0, ptr(sums),
                        2 * Ci if fuse32 else 0, dx.data_ptr(), ptr(residual),
                        *_hconv_split(K, N, OH, OW, 2 * Co, Ci, 9, dy.device), st,
                        bnb.args() if fuse32 else _NOBNB):
            _H3_F32_STATS["dgrad"] += 1
            if fuse32:
                _H3_F32_STATS["dgrad_bnb"] += 1
                dx._bnb = (bnb.bn, slab, rows, sums)
            return dx
    g2 = K.gemm_g2f if f32 else K.gemm_g2
    fuse = (bnb is not None and fusion.BNB and not bnb.pooled and not f32 and not empty_class and bnb.x.dtype == BF16
            and tuple(bnb.x.shape) == (N, Ci, H, W))
    if not f32 and len(classes) == 1 and not empty_class and route == K.ROUTE_HALO and \
            len(classes[0][4]) == KH * KW:
        slab = sums = None
        rows = 0
        if fuse:
            rows = K.hconv_stat_rows(N, H, W, Co, Ci, len(classes[0][4]), 0)
            slab = _empty((rows, 2, Ci), F32, dy.device)
            sums = _empty((2 * Ci,), F32, dy.device)  # zeroed in-kernel
        K.hconv(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _nbytes(dy), _nbytes(wt), N, OH, OW, Co, Ci, KH * KW * Co,
                [(t[0], t[1], t[3]) for t in classes[0][4]], 0, ptr(residual), ptr(slab), 0, ptr(sums),
                2 * Ci if fuse else 0, bnb.args() if fuse else _NOBNB, 0, 0,
                *_hconv_split(K, N, OH, OW, Co, Ci, len(classes[0][4]), dy.device), st)
        if fuse:
            dx._bnb = (bnb.bn, slab, rows, sums)
        return dx
    if (not f32 and fusion.G2_GROUP and len(classes) > 1 and len({(c[2], c[3]) for c in classes}) == 1
            and (N * classes[0][2] * classes[0][3]) % 128 == 0):
        # all stride phases in ONE grouped launch (gemm_g2 row classes): no per-phase launch
        # boundaries, and the grid covers the whole dgrad instead of a quarter of it
        GH, GW = classes[0][2], classes[0][3]
        M = len(classes) * N * GH * GW
        taps_all, groups = [], []
        for ry, rx, _, _, taps in classes:
            groups.append((len(taps_all), len(taps), ry, rx))
            taps_all += taps
        rows = K.gemm_g2_stat_rows(M, Ci) if fuse else 0
        slab = _empty((rows, 2, Ci), F32, dy.device) if fuse else None
        sums = _empty((2 * Ci,), F32, dy.device) if fuse else None
        K.gemm_g2_grouped(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _nbytes(dy), _nbytes(wt), M, Ci, Co, OH, OW,
                          GH, GW, 1, 1, taps_all, KH * KW * Co, Ci, H, W, sh, sw, 0, 0, 0, ptr(residual), ptr(slab), 0,
                          ptr(sums), 2 * Ci if fuse else 0, bnb.args() if fuse else _NOBNB, st, groups)
        if fuse:
            dx._bnb = (bnb.bn, slab, rows, sums)
        return dx
    if not f32 and route == K.ROUTE_G1S and not empty_class and len(classes) == 1:
        # streaming 1x1 data gradient (g1s.hip), backward-BatchNorm fusion in its epilogue
        rows = K.g1s_rows(N * H * W, Ci, Co, 2 if fuse else 0)
        if rows:
            slab = _empty((rows, 2, Ci), F32, dy.device) if fuse else None
            sums = _empty((2 * Ci,), F32, dy.device) if fuse else None
            K.g1s(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N * H * W, Ci, Co, H, W, H, W, 1, 0, ptr(residual),
                  ptr(slab), 0, ptr(sums), 2 * Ci if fuse else 0, bnb.args() if fuse else _NOBNB, 2 if fuse else 0, st)
            if fuse:
                dx._bnb = (bnb.bn, slab, rows, sums)
            return dx
    crow = [K.gemm_g2_stat_rows(N * GH * GW, Ci) if fuse else 0 for _, _, GH, GW, _ in classes]
    rows = sum(crow)
    slab = _empty((rows, 2, Ci), F32, dy.device) if fuse else None
    sums = _empty((2 * Ci,), F32, dy.device) if fuse else None
    r0 = 0
    for k, (ry, rx, GH, GW, taps) in enumerate(classes):
        sp = slab.data_ptr() + r0 * 2 * Ci * 4 if fuse else 0
        zp = ptr(sums) if (fuse and k == 0) else 0
        g2(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), _nbytes(dy), _nbytes(wt), N * GH * GW, Ci, Co, OH, OW,
           GH, GW, 1, 1, taps, KH * KW * Co, Ci, H, W, sh, sw, ry, rx, 0, ptr(residual), sp, 0, zp,
           2 * Ci if zp else 0, bnb.args() if fuse else _NOBNB, st)
        r0 += crow[k]
    if fuse:
        dx._bnb = (bnb.bn, slab, rows, sums)
    return dx


def conv2d_wgrad(dy, x, w_shape, stride, pad, grad_w, grad_b=None):
    """grad_w (+)= dW, grad_b (+)= sum(dy): split-K MFMA GEMM + fp32 slab reduce (beta = 1).

    ``x`` may carry zero-padded channels (RGB stem); the padded columns are dropped on reduce.
    """
    if _CONV_ALGO == "im2col" and x.shape[1] == w_shape[1] and _im2col_ok(w_shape[1], w_shape[0]):
        return conv2d_wgrad_im2col(dy, x, w_shape, stride, pad, grad_w, grad_b)
    K = kernels()
    N, Cx, H, W = x.shape
    Co, Ci, KH, KW = w_shape
    OH, OW = dy.shape[2], dy.shape[3]
    P = N * OH * OW
    st = stream_ptr()
    taps = [(ky - pad[0], kx - pad[1]) for ky in range(KH) for kx in range(KW)]
    hw_ok = (Cx == Ci and tuple(stride) == (1, 1) and (OH, OW) == (H, W)
             and 1 < len(taps) <= 9 and all(abs(a) <= 1 and abs(b) <= 1 for a, b in taps)
             and K.hwgrad_supported(N, H, W, Ci, Co, len(taps)))
    if dy.dtype == F32 and hw_ok and _f32_concat_ok(Ci, Co):
        # split-precision fp32 on the halo wgrad: three (dY, X) channel windows of the split rows
        # (dyh, xh), (dyh, xl), (dyl, xh); the bias partial is sum(dyh) + sum(dyl)
        dys, xs = act_split3(dy), act_split3(x)
        Ng = KH * KW * Ci
        splits = K.hwgrad_splits(N, H, W, Ci, Co)
        slab = _empty((3 * splits, Co, Ng), F32, x.device)
        bslab = _empty((3 * splits, Co), F32, x.device) if grad_b is not None else None
        K.hwgrad(dys.data_ptr(), xs.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dys), _nbytes(xs), N, H, W, Ci,
                 Co, taps, splits, 3 * Co, 3 * Ci, [(0, 0, 1), (0, Ci, 0), (Co, 0, 1)], st)
        _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, 3 * splits, st)
        return
    if (dy.dtype == F32 and _HW_F32 and Cx == Ci and (KH, KW, *stride, *pad) == (3, 3, 1, 1, 1, 1)
            and (OH, OW) == (H, W) and K.hwgrad_f32_supported(N, H, W, Ci, Co)):
        Ng = 9 * Ci
        splits = K.hwgrad_f32_splits(N, H, W, Ci, Co)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        K.hwgrad_f32(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy), _nbytes(x), N, H, W,
                     Ci, Co, splits, st)
        _H3_F32_STATS["wgrad"] += 1
        _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
        return
    if dy.dtype == F32:
        assert x.dtype == F32 and Cx == Ci
        Ng = KH * KW * Ci
        splits = K.gemm_t2f_splits(Co, Ng, P)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        taps = [(ky - pad[0], kx - pad[1]) for ky in range(KH) for kx in range(KW)]
        K.gemm_t2f(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), Co, Ng, P, Co, Ci, H, W, OH, OW,
                   stride[0], stride[1], taps, splits, st)
        assert grad_w.is_contiguous(memory_format=CL) or KH * KW == 1 or Ci == 1
        _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
        return
    # the shared routing table (csrc/kernels/conv_route.cpp, also used by the C++ host API)
    route = (K.conv_wgrad_route(N, Ci, H, W, Co, KH, KW, stride[0], stride[1], pad[0], pad[1], OH, OW, -1)
             if Cx == Ci else K.ROUTE_GEMM_G2)
    _rec("wgrad", x=(N, Ci, H, W), xpad=Cx, w=(Co, Ci, KH, KW), stride=tuple(stride), pad=tuple(pad),
         bias=grad_b is not None, route=int(route))
    if route == K.ROUTE_HALO_S2 and fusion.HWGRAD_S2:
        # stride-2 halo wgrad: the 64-pixel tile's (2 TH + 1) x (2 TW + 1) input halo staged once for 9 taps
        Ng = 9 * Ci
        splits = K.hwgrad_s2_splits(N, OH, OW, Ci, Co)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        K.hwgrad_s2(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy), _nbytes(x), N, OH, OW, Ci,
                    Co, splits, st)
        _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
        return
    if route == K.ROUTE_HALO:
        # halo-tiled wgrad: X read ~1.4x instead of once per tap
        Ng = KH * KW * Ci
        splits = K.hwgrad_splits(N, H, W, Ci, Co)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        K.hwgrad(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy), _nbytes(x), N, H, W, Ci, Co,
                 taps, splits, Co, Ci, [], st)
        _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
        return
    if _g2_ok(Cx, Co) and P < (1 << 24):
        Ng = KH * KW * Cx
        splits = K.gemm_t2_splits(Co, Ng, P)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        taps = [(ky - pad[0], kx - pad[1]) for ky in range(KH) for kx in range(KW)]
        K.gemm_t2(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy), _nbytes(x), Co, Ng, P, Co, Cx,
                  H, W, OH, OW, stride[0], stride[1], taps, splits, st)
        if Cx == Ci:
            _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
            return
        tmp = _empty((Co, KH, KW, Cx), F32, x.device)
        K.splitk_reduce(slab.data_ptr(), tmp.data_ptr(), Co * Ng, splits, 0, st)
        if grad_w.is_contiguous(memory_format=CL):
            K.rows_copy(1, tmp.data_ptr(), Cx, grad_w.data_ptr(), Ci, Co * KH * KW, Ci, st)
        else:
            grad_w.add_(tmp[..., :Ci].permute(0, 3, 1, 2))
        if grad_b is not None:
            K.splitk_reduce(bslab.data_ptr(), grad_b.data_ptr(), Co, splits, 1, st)
        return
    Ng = KH * KW * Ci
    splits = K.gemm_tn_splits(Co, Ng, P)
    slab = _empty((splits, Co, Ng), F32, x.device)
    bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
    K.gemm_tn(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), ptr(bslab), Co, Ng, P, CONV_FWD,
              N, H, W, Ci, OH, OW, KH, KW, stride[0], stride[1], pad[0], pad[1], 0, splits, st)
    assert grad_w.is_contiguous(memory_format=CL) or KH * KW == 1 or Ci == 1
    _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)
