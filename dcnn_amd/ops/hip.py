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
import threading

import torch

from ..runtime import arena as _arena
from ._ext import dt_code, kernels, ptr, stream_ptr

CL = torch.channels_last
F32 = torch.float32
BF16 = torch.bfloat16

# backward-BN epilogue fusion operands (api.h BnbArgs): (y, x, mean, istd) pointers, 0 = off
_NOBNB = (0, 0, 0, 0)

# gather modes of gemm_nt
PLAIN, CONV_FWD, CONV_DGRAD = 0, 1, 2


def _empty(shape, dtype, device, cl=False):
    """Per-step buffer (activation, statistics slab, workspace): the native activation arena of
    the running step (runtime/arena.py), else PyTorch's allocator. ``cl``: NHWC strides."""
    return _arena.empty(shape, dtype, device, cl)


def _empty_like(x):
    """Per-step buffer shaped and laid out (dense or channels_last) like x."""
    cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=CL)
    return _arena.empty(x.shape, x.dtype, x.device, cl)


def _check_act(x: torch.Tensor, what: str):
    if not x.is_cuda:
        raise ValueError(f"{what}: expected a GPU tensor")
    if x.dim() == 4 and not x.is_contiguous(memory_format=CL):
        raise ValueError(f"{what}: expected channels_last (NHWC) memory layout")


# ---- conv call recorder (tests/test_gpu_geometry.py): every conv2d_fwd / dgrad / wgrad call's
# shapes, epilogue options and routing-table decision, so a test can replay exactly the (kernel,
# shape, epilogue) tuples a model's training step launches against an fp32 reference
_RECORD = None


class record_convs:
    """``with record_convs() as calls:`` appends one dict per conv call made inside the block."""

    def __enter__(self):
        global _RECORD
        self._prev, self.calls = _RECORD, []
        _RECORD = self.calls
        return self.calls

    def __exit__(self, *exc):
        global _RECORD
        _RECORD = self._prev
        return False


def _rec(op, **kw):
    if _RECORD is not None:
        _RECORD.append(dict(op=op, **kw))


def to_act(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Bring a (N,C,H,W) tensor into the GPU activation format: NHWC memory, compute dtype."""
    if x.dim() == 4 and x.dtype == dtype and x.is_contiguous(memory_format=CL):
        return x
    if x.dim() == 4 and x.dtype == F32 and x.is_contiguous():
        # fused NCHW fp32 -> NHWC (bf16|fp32) conversion kernel (network input path)
        N, C, H, W = x.shape
        y = _empty((N, C, H, W), dtype, x.device, True)
        kernels().nchw_to_nhwc(dt_code(dtype), x.data_ptr(), y.data_ptr(), N, C, H * W, stream_ptr())
        return y
    return x.to(dtype=dtype).contiguous(memory_format=CL)


def nchw_nhwc(x: torch.Tensor, to_nhwc: bool) -> torch.Tensor:
    """Physical layout change of a 4-D GPU activation (the NCHW-order Flatten of a spatial map):
    NCHW-contiguous -> channels_last (to_nhwc) or back, one transpose kernel per call (fp32 / bf16)."""
    N, C, H, W = x.shape
    if to_nhwc:
        assert x.is_contiguous()
        y = _empty((N, C, H, W), x.dtype, x.device, True)
        rows, cols = C, H * W
    else:
        assert x.is_contiguous(memory_format=CL)
        y = _empty((N, C, H, W), x.dtype, x.device, False)
        rows, cols = H * W, C
    if x.dtype == F32:
        kernels().transpose_batched(x.data_ptr(), y.data_ptr(), N, rows, cols, stream_ptr())
    else:
        assert x.element_size() == 2
        kernels().transpose_batched16(x.data_ptr(), y.data_ptr(), N, rows, cols, stream_ptr())
    return y


def conv_out_hw(H, W, kh, kw, sh, sw, ph, pw):
    return (H + 2 * ph - kh) // sh + 1, (W + 2 * pw - kw) // sw + 1


# ------------------------------------------------------------------------------ conv / dense
def _nbytes(t):
    return t.numel() * t.element_size()


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


def _g2_ok(Cs, N):
    return Cs % 8 == 0 and N % 8 == 0



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
_HCONV_1X1 = True


def _hconv_ok(N, OH, OW, H, W, sh, sw, Cs, Co, taps, wop, split3=False):
    """Halo-tiled direct conv applies to stride-1 'same' convs with a 1-pixel reach (3x3/pad 1
    forward and its dgrad) on 64-multiple channel counts. ``split3``: the caller is a 3 x bf16
    fp32 concat path (Cs = 3 x the real channels): 1x1 convs stay on the exact fp32 GEMM there."""
    if (sh, sw) != (1, 1) or (OH, OW) != (H, W) or len(taps) > 9:
        return False
    if any(abs(t[0]) > 1 or abs(t[1]) > 1 for t in taps):
        return False
    if len(taps) == 1 and not (_HCONV_1X1 and not split3 and Cs >= 1024 and (N * OH * OW // 64) * (Co // 64) < 256):
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
_H3_F32_STATS = {"fwd": 0, "dgrad": 0, "wgrad": 0}


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
    if route == K.ROUTE_HALO and KH * KW == 1 and not _HCONV_1X1:
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




def stem_ok(x, w_shape, stride, pad):
    """The RGB stem kernels (stem.hip) take this conv: fp32 NCHW input, 3x3 s1 p1, Ci <= 4."""
    if x.dtype != F32 or not x.is_contiguous() or x.dim() != 4:
        return False
    Co, Ci, KH, KW = w_shape
    N, C, H, W = x.shape
    return ((KH, KW) == (3, 3) and tuple(stride) == (1, 1) and tuple(pad) == (1, 1) and C == Ci
            and kernels().stem_supported(N, Ci, H, W, Co))


def stem_conv_fwd(x, w, bias=None, stats=False):
    """3x3/s1/p1 conv of the fp32 NCHW network input (Ci <= 4) -> bf16 NHWC, optionally with the
    BatchNorm partial statistics (same ``(slab, rows, sums)`` contract as :func:`conv2d_fwd`).
    ``w``: (Co, Ci, 3, 3) fp32 or bf16, any strides. One pass: no layout/pad kernel."""
    N, Ci, H, W = x.shape
    Co = w.shape[0]
    K = kernels()
    _rec("stem_fwd", x=(N, Ci, H, W), w=(Co, Ci, 3, 3), stats=bool(stats), bias=bias is not None, route=-1)
    y = _empty((N, Co, H, W), BF16, x.device, True)
    slab = sums = None
    rows = 0
    if stats:
        rows = K.stem_tiles(N, H, W)
        slab = _empty((rows, 3, Co), F32, x.device)
        sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
    assert w.dtype in (F32, BF16) and tuple(w.shape) == (Co, Ci, 3, 3)
    K.stem_fwd(x.data_ptr(), w.data_ptr(), int(w.dtype == BF16), list(w.stride()), ptr(bias), y.data_ptr(),
               ptr(slab), ptr(sums), 2 * Co if stats else 0, N, Ci, H, W, Co, stream_ptr())
    return y, ((slab, rows, sums) if stats else None)


def stem_conv_wgrad(dy, x, grad_w, grad_b=None):
    """grad_w += dW, grad_b += sum(dy) of :func:`stem_conv_fwd` (dy: bf16 NHWC)."""
    N, Ci, H, W = x.shape
    Co = dy.shape[1]
    K = kernels()
    _rec("stem_wgrad", x=(N, Ci, H, W), w=(Co, Ci, 3, 3), bias=grad_b is not None, route=-1)
    dy = dy.contiguous(memory_format=CL)
    assert dy.dtype == BF16 and tuple(dy.shape) == (N, Co, H, W)
    assert grad_w.is_contiguous() or grad_w.is_contiguous(memory_format=CL), "dense fp32 weight gradient"
    blocks = K.stem_wgrad_blocks(N, H, W)
    n = Co * Ci * 9
    slab = _empty((blocks, n), F32, x.device)
    bslab = _empty((blocks, Co), F32, x.device) if grad_b is not None else None
    st = stream_ptr()
    K.stem_wgrad(x.data_ptr(), dy.data_ptr(), slab.data_ptr(), ptr(bslab), list(grad_w.stride()), N, Ci, H, W, Co,
                 blocks, st)
    _reduce_wb(K, slab, grad_w, n, bslab, grad_b, Co, blocks, st)


def to_act_padded(x, cp):
    """(N,C,H,W) -> NHWC bf16 with channels zero-padded to cp (RGB stem: 3 -> 8) so the stem
    conv runs on the vectorised MFMA path. One HIP pass from an NCHW fp32 input."""
    N, C, H, W = x.shape
    y = _empty((N, cp, H, W), BF16, x.device, True)
    src = x if (x.dtype == F32 and x.is_contiguous()) else x.float().contiguous()
    kernels().nchw_to_nhwc_pad(dt_code(BF16), src.data_ptr(), y.data_ptr(), N, C, cp, H * W, stream_ptr())
    return y


def pad_weight_channels(w, cp, out=None):
    """(Co,Ci,KH,KW) -> bf16 [Co][KH][KW][cp] operand, zero-padded input channels. ``out``: a
    previous result to refresh in place (one copy of the real channels, padding already zero)."""
    Co, Ci, KH, KW = w.shape
    if out is None or tuple(out.shape) != (Co, KH, KW, cp) or out.device != w.device:
        out = _arena.persistent((Co, KH, KW, cp), BF16, w.device, zero=True)  # cached by the layer
    if w.dtype == BF16 and w.is_contiguous(memory_format=CL):
        # the layer's bf16 shadow: [Co*KH*KW] rows of Ci channels into rows of cp (one HIP pass)
        kernels().rows_copy(0, w.data_ptr(), Ci, out.data_ptr(), cp, Co * KH * KW, Ci, stream_ptr())
    else:
        out[..., :Ci] = w.permute(0, 2, 3, 1).to(BF16)
    return out


def conv_weight_t(w, out=None, dtype=BF16):
    """(Co,Ci,KH,KW) channels_last weight -> [Ci][KH][KW][Co] dgrad operand (bf16, or fp32 for
    the fp32 compute path)."""
    Co, Ci, KH, KW = w.shape
    if dtype == F32:
        src = w if (w.dtype == F32 and (w.is_contiguous(memory_format=CL) or KH * KW == 1 or Ci == 1)) \
            else w.float().contiguous(memory_format=CL)
        if out is None:
            out = _empty((Ci, KH, KW, Co), F32, w.device)
        kernels().conv_weight_transpose_f32(src.data_ptr(), out.data_ptr(), Co, KH * KW, Ci, stream_ptr())
        return out
    if out is None:
        out = _empty((Ci, KH, KW, Co), BF16, w.device)
    kernels().conv_weight_transpose(dt_code(w.dtype), w.data_ptr(), out.data_ptr(), Co, KH * KW, Ci, stream_ptr())
    return out


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


def _im2col_ok(Ci, Co):
    return Ci % 8 == 0 and Co % 8 == 0


def _geom(N, H, W, C, OH, OW, KH, KW, stride, pad):
    return (N, H, W, C, OH, OW, KH, KW, stride[0], stride[1], pad[0], pad[1])


def im2col_nhwc(x, KH, KW, stride, pad):
    """(N,C,H,W) channels_last -> column matrix [N*OH*OW][KH*KW*C] (tap-major, zero padding)."""
    _check_act(x, "im2col_nhwc.x")
    N, C, H, W = x.shape
    OH, OW = conv_out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    col = _empty((N * OH * OW, KH * KW * C), x.dtype, x.device)
    kernels().im2col_nhwc(dt_code(x.dtype), x.data_ptr(), col.data_ptr(), *_geom(N, H, W, C, OH, OW, KH, KW, stride, pad),
                          stream_ptr())
    return col


def col2im_nhwc(col, x_shape, KH, KW, stride, pad, *, residual=None, chan_major=False):
    """Sum the column matrix back onto (N,C,H,W) channels_last (+ residual); ``chan_major``: the
    columns are ordered (c, ky, kx) instead of (ky, kx, c)."""
    N, C, H, W = x_shape
    OH, OW = conv_out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    assert tuple(col.shape) == (N * OH * OW, KH * KW * C) and col.is_contiguous()
    x = _empty((N, C, H, W), col.dtype, col.device, True)
    if residual is not None:
        assert tuple(residual.shape) == (N, C, H, W) and residual.dtype == col.dtype
        assert residual.is_contiguous(memory_format=CL)
    kernels().col2im_nhwc(dt_code(col.dtype), col.data_ptr(), x.data_ptr(), ptr(residual),
                          *_geom(N, H, W, C, OH, OW, KH, KW, stride, pad), int(chan_major), stream_ptr())
    return x


def conv2d_fwd_im2col(x, w, bias, stride, pad, *, stats=False, residual=None, relu=False):
    """:func:`conv2d_fwd` by explicit im2col + one plain MFMA GEMM (same fused epilogue: bias,
    residual, ReLU, BatchNorm partial statistics; same return contract)."""
    K = kernels()
    N, Ci, H, W = x.shape
    Co, _, KH, KW = w.shape
    assert w.dtype == x.dtype and w.is_contiguous(memory_format=CL)
    col = im2col_nhwc(x, KH, KW, stride, pad)
    M, Kc = col.shape
    OH, OW = conv_out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    if residual is not None:
        assert tuple(residual.shape) == (N, Co, OH, OW) and residual.is_contiguous(memory_format=CL)
    f32 = x.dtype == F32
    y = _empty((N, Co, OH, OW), x.dtype, x.device, True)
    slab, rows, sums = None, 0, None
    if stats:
        rows = (K.gemm_g2f_stat_rows if f32 else K.gemm_g2_stat_rows)(M, Co)
        slab = _empty((rows, 3, Co), F32, x.device)
        sums = _empty((2 * Co,), F32, x.device)  # zeroed in-kernel
    (K.gemm_g2f if f32 else K.gemm_g2)(col.data_ptr(), w.data_ptr(), y.data_ptr(), _nbytes(col), _nbytes(w), M, Co,
                                       Kc, 1, 1, 1, 1, 1, 1, [(0, 0, 0, 0)], Kc, Co, 1, 1, 1, 1, 0, 0, ptr(bias),
                                       ptr(residual), ptr(slab), int(relu), ptr(sums), 2 * Co if stats else 0, _NOBNB,
                                       stream_ptr())
    return y, ((slab, rows, sums) if stats else None)


def conv2d_dgrad_im2col(dy, wt, x_shape, stride, pad, *, residual=None):
    """:func:`conv2d_dgrad` by a plain GEMM into a channel-major column matrix
    (dy [M][Co] . wt[Ci*KH*KW][Co]^T) and a gather col2im (+ residual)."""
    K = kernels()
    N, Ci, H, W = x_shape
    Ci2, KH, KW, Co = wt.shape
    assert Ci2 == Ci and dy.shape[1] == Co and wt.dtype == dy.dtype and wt.is_contiguous()
    M = dy.shape[0] * dy.shape[2] * dy.shape[3]
    Nc = Ci * KH * KW
    colg = _empty((M, Nc), dy.dtype, dy.device)
    (K.gemm_g2f if dy.dtype == F32 else K.gemm_g2)(dy.data_ptr(), wt.data_ptr(), colg.data_ptr(), _nbytes(dy),
                                                   _nbytes(wt), M, Nc, Co, 1, 1, 1, 1, 1, 1, [(0, 0, 0, 0)], Co, Nc,
                                                   1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, _NOBNB, stream_ptr())
    return col2im_nhwc(colg, x_shape, KH, KW, stride, pad, residual=residual, chan_major=True)


def conv2d_wgrad_im2col(dy, x, w_shape, stride, pad, grad_w, grad_b=None):
    """:func:`conv2d_wgrad` as dW[Co][KH*KW*Ci] = dy^T . im2col(x): split-K MFMA GEMM + slab reduce."""
    K = kernels()
    Co, Ci, KH, KW = w_shape
    col = im2col_nhwc(x, KH, KW, stride, pad)
    P, Ng = col.shape
    assert dy.shape[0] * dy.shape[2] * dy.shape[3] == P and dy.shape[1] == Co
    assert grad_w.is_contiguous(memory_format=CL) or KH * KW == 1 or Ci == 1
    st = stream_ptr()
    if dy.dtype == F32:
        splits = K.gemm_t2f_splits(Co, Ng, P)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        K.gemm_t2f(dy.data_ptr(), col.data_ptr(), slab.data_ptr(), ptr(bslab), Co, Ng, P, Co, Ng, 1, 1, 1, 1, 1, 1,
                   [(0, 0)], splits, st)
    else:
        splits = K.gemm_t2_splits(Co, Ng, P)
        slab = _empty((splits, Co, Ng), F32, x.device)
        bslab = _empty((splits, Co), F32, x.device) if grad_b is not None else None
        K.gemm_t2(dy.data_ptr(), col.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy), _nbytes(col), Co, Ng, P,
                  Co, Ng, 1, 1, 1, 1, 1, 1, [(0, 0)], splits, st)
    _reduce_wb(K, slab, grad_w, Co * Ng, bslab, grad_b, Co, splits, st)


class BnbRequest:
    """Backward-BatchNorm fusion request handed to a gradient producer (api.h ``BnbArgs``).

    ``bn`` is the consuming BatchNorm layer; ``y`` its (ReLU) output used as the mask (None: no
    ReLU was fused), ``x`` its input, ``mean``/``istd`` its saved batch statistics. A producer
    that honours the request returns dy' = dy * (y > 0) with ``dy'._bnb = (bn, slab, rows, sums)``
    attached: per-tile (sum dy', sum dy' * xhat) rows and the zeroed [2][C] sums to reduce into.
    """
    __slots__ = ("bn", "y", "x", "mean", "istd", "pooled")

    def __init__(self, bn, y, x, mean, istd, pooled=False):
        # pooled: the BatchNorm's forward fused ReLU + max-pool (no full-resolution y; only the
        # max-pool backward, masking with the pooled value, can honour the request)
        self.bn, self.y, self.x, self.mean, self.istd, self.pooled = bn, y, x, mean, istd, pooled

    def args(self):
        return (ptr(self.y), self.x.data_ptr(), self.mean.data_ptr(), self.istd.data_ptr())


# fusion / batching choices, module constants so the GPU tests can compare each against the
# unfused path it replaces
_G2_GROUP = True  # strided dgrad phases in one launch
_BNB = True  # backward-BatchNorm fusion (ReLU mask + statistics) into the producing dgrad epilogue
_BN_DUAL = True  # projection-shortcut BatchNorm pairs in one pass
_DEFER_REDUCE = True  # one batched split-K weight-gradient reduce per backward


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
    fuse_req = bnb is not None and _BNB and not bnb.pooled and not f32 and bnb.x.dtype == BF16 \
        and tuple(bnb.x.shape) == (N, Ci, H, W)
    # the shared routing table (csrc/kernels/conv_route.cpp, also used by the C++ host API)
    route = K.conv_dgrad_route(N, Ci, H, W, Co, KH, KW, sh, sw, ph, pw, OH, OW, 2 if fuse_req else 0) \
        if not f32 else K.ROUTE_GEMM_G2
    if route == K.ROUTE_HALO and KH * KW == 1 and not _HCONV_1X1:
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
    if (not f32 and empty_class and len(classes) > 1 and _G2_GROUP and len(allc) <= 4
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
        # exact fp32 data gradient on the persistent halo conv (transposed weights, reversed taps)
        if K.hconv3_f32(dy.data_ptr(), wt.data_ptr(), _nbytes(dy), _nbytes(wt), N, OH, OW, Co, Ci, KH * KW * Co,
                        [(t[0], t[1], t[3]) for t in classes[0][4]], 0, 0, 0, 0, 0, dx.data_ptr(), ptr(residual),
                        *_hconv_split(K, N, OH, OW, 2 * Co, Ci, 9, dy.device), st):
            _H3_F32_STATS["dgrad"] += 1
            return dx
    g2 = K.gemm_g2f if f32 else K.gemm_g2
    fuse = (bnb is not None and _BNB and not bnb.pooled and not f32 and not empty_class and bnb.x.dtype == BF16
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
    if (not f32 and _G2_GROUP and len(classes) > 1 and len({(c[2], c[3]) for c in classes}) == 1
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


class _DeferredReduce:
    """Split-K weight-gradient reductions queued during a model backward and launched together
    (``multi_splitk_reduce``: one kernel for the whole queue instead of one per layer, ~26 for
    ResNet-18). The slabs stay referenced until the flush; with 288 GB of HBM per GPU holding
    every layer's slab for one backward (< 2 GB for ResNet-18 at batch 256) is the cheap side of
    the trade. Active between ``begin()`` / ``end()`` (Sequential.prepare_backward /
    finish_backward); gradient consumers inside that window (the data-parallel bucket
    all-reduce) call ``flush()`` first. Outside it every reduction runs immediately."""

    def __init__(self):
        self.active = False
        self.pending = []  # (slab, out, n, splits) — tensors kept alive until the launch
        self.pending_bytes = 0

    def begin(self):
        self.active = _DEFER_REDUCE

    def add(self, slab, out, n, splits):
        self.pending.append((slab, out, int(n), int(splits)))
        self.pending_bytes += int(n) * int(splits) * 4
        # a queue larger than the last-level cache would read its first slabs back from HBM:
        # launch once the pending slabs reach the threshold
        if self.pending_bytes >= _DEFER_REDUCE_BYTES:
            self.flush()

    def flush(self):
        if self.pending and _TRACE_REDUCE:
            import sys
            print(f"[splitk_reduce] {len(self.pending)} slabs, {self.pending_bytes / 2**20:.1f} MiB: "
                  + " ".join(f"{t[2]}x{t[3]}" for t in self.pending), file=sys.stderr)
        if self.pending:
            kernels().multi_splitk_reduce([(t[0].data_ptr(), t[1].data_ptr(), t[2], t[3]) for t in self.pending],
                                          stream_ptr())
            self.pending.clear()
            self.pending_bytes = 0

    def end(self):
        self.flush()
        self.active = False


_TRACE_REDUCE = os.environ.get("DCNN_TRACE_REDUCE", "0") == "1"  # print each batched reduce's slabs
_DEFER_REDUCE_BYTES = 1 << 50  # (one batched reduce per backward)
_tls = threading.local()


class _ThreadReducer:
    """``grad_reducer``: the calling thread's :class:`_DeferredReduce` (a pipeline stage's
    backward on its own thread and stream must not flush another stage's queue)."""

    def _get(self):
        r = getattr(_tls, "reducer", None)
        if r is None:
            r = _tls.reducer = _DeferredReduce()
        return r

    def __getattr__(self, k):
        return getattr(self._get(), k)


grad_reducer = _ThreadReducer()

def _dense(t):
    """A gradient tensor whose storage is exactly its numel() elements (any dim order)."""
    return t.is_contiguous() or t.is_contiguous(memory_format=CL)


def _reduce_wb(K, slab, grad_w, n, bslab, grad_b, nb, splits, st):
    """grad_w += sum over splits of slab, grad_b += sum of bslab — one launch for both (or
    queued on :data:`grad_reducer` inside a model backward)."""
    if grad_reducer.active and _dense(grad_w) and (grad_b is None or grad_b.is_contiguous()):
        grad_reducer.add(slab, grad_w, n, splits)
        if grad_b is not None:
            grad_reducer.add(bslab, grad_b, nb, splits)
        return
    if grad_b is None:
        K.splitk_reduce(slab.data_ptr(), grad_w.data_ptr(), n, splits, 1, st)
    else:
        K.splitk_reduce2(slab.data_ptr(), grad_w.data_ptr(), n, bslab.data_ptr(), grad_b.data_ptr(), nb, splits, 1, st)


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


def dense_fwd(x2d, w2d, bias):
    """y[N,Out] = x[N,In] . w[Out,In]^T + b   (bf16 in/out, fp32 accumulate)."""
    N, In = x2d.shape
    Out = w2d.shape[0]
    if x2d.dtype == F32:
        y = _empty((N, Out), F32, x2d.device)
        kernels().gemm_g2f(x2d.data_ptr(), w2d.data_ptr(), y.data_ptr(), _nbytes(x2d), _nbytes(w2d), N, Out, In, 1, 1,
                           1, 1, 1, 1, [(0, 0, 0, 0)], In, Out, 1, 1, 1, 1, 0, 0, ptr(bias), 0, 0, 0, 0, 0, _NOBNB,
                           stream_ptr())
        return y
    y = _empty((N, Out), BF16, x2d.device)
    if _g2_ok(In, Out):
        kernels().gemm_g2(x2d.data_ptr(), w2d.data_ptr(), y.data_ptr(), _nbytes(x2d), _nbytes(w2d), N, Out, In, 1, 1,
                          1, 1, 1, 1, [(0, 0, 0, 0)], In, Out, 1, 1, 1, 1, 0, 0, ptr(bias), 0, 0, 0, 0, 0, _NOBNB,
                          stream_ptr())
        return y
    kernels().gemm_nt(x2d.data_ptr(), w2d.data_ptr(), y.data_ptr(), N, Out, In, In, In, Out, PLAIN,
                      0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0, ptr(bias), 0, 0, 0, 0, stream_ptr())
    return y


def dense_dgrad(dy2d, wt2d):
    """dx[N,In] = dy[N,Out] . w[Out,In]   with wt2d = w^T stored [In][Out]."""
    N, Out = dy2d.shape
    In = wt2d.shape[0]
    if dy2d.dtype == F32:
        dx = _empty((N, In), F32, dy2d.device)
        kernels().gemm_g2f(dy2d.data_ptr(), wt2d.data_ptr(), dx.data_ptr(), _nbytes(dy2d), _nbytes(wt2d), N, In, Out,
                           1, 1, 1, 1, 1, 1, [(0, 0, 0, 0)], Out, In, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, _NOBNB,
                           stream_ptr())
        return dx
    dx = _empty((N, In), BF16, dy2d.device)
    if _g2_ok(Out, In):
        kernels().gemm_g2(dy2d.data_ptr(), wt2d.data_ptr(), dx.data_ptr(), _nbytes(dy2d), _nbytes(wt2d), N, In, Out, 1,
                          1, 1, 1, 1, 1, [(0, 0, 0, 0)], Out, In, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, _NOBNB,
                          stream_ptr())
        return dx
    kernels().gemm_nt(dy2d.data_ptr(), wt2d.data_ptr(), dx.data_ptr(), N, In, Out, Out, Out, In, PLAIN,
                      0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, stream_ptr())
    return dx


def dense_wgrad(dy2d, x2d, grad_w, grad_b=None):
    K = kernels()
    N, Out = dy2d.shape
    In = x2d.shape[1]
    st = stream_ptr()
    if dy2d.dtype == F32:
        splits = K.gemm_t2f_splits(Out, In, N)
        slab = _empty((splits, Out, In), F32, x2d.device)
        bslab = _empty((splits, Out), F32, x2d.device) if grad_b is not None else None
        K.gemm_t2f(dy2d.data_ptr(), x2d.data_ptr(), slab.data_ptr(), ptr(bslab), Out, In, N, Out, In, 1, 1, 1, 1,
                   1, 1, [(0, 0)], splits, st)
    elif _g2_ok(In, Out):
        splits = K.gemm_t2_splits(Out, In, N)
        slab = _empty((splits, Out, In), F32, x2d.device)
        bslab = _empty((splits, Out), F32, x2d.device) if grad_b is not None else None
        K.gemm_t2(dy2d.data_ptr(), x2d.data_ptr(), slab.data_ptr(), ptr(bslab), _nbytes(dy2d), _nbytes(x2d), Out, In,
                  N, Out, In, 1, 1, 1, 1, 1, 1, [(0, 0)], splits, st)
    else:
        splits = K.gemm_tn_splits(Out, In, N)
        slab = _empty((splits, Out, In), F32, x2d.device)
        bslab = _empty((splits, Out), F32, x2d.device) if grad_b is not None else None
        K.gemm_tn(dy2d.data_ptr(), x2d.data_ptr(), slab.data_ptr(), ptr(bslab), Out, In, N, PLAIN,
                  0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0, In, splits, st)
    _reduce_wb(K, slab, grad_w, Out * In, bslab, grad_b, Out, splits, st)


# ------------------------------------------------------------------------------ batch norm
def _rc(x):
    N, C, H, W = x.shape
    return N * H * W, C


_tickets = {}


def _ticket(device, C, slot="stat"):
    """Per-(stream, device, user) ticket words of the ticketed reductions (bn_stat_reduce, the
    loss): zeroed once, every launch leaves them zeroed again, and launches on one stream never
    overlap."""
    key = (stream_ptr(), device.index, slot)
    t = _tickets.get(key)
    need = (C + 63) // 64
    if t is None or t.numel() < need:
        t = _arena.persistent((max(need, 64),), torch.int32, torch.device(device), zero=True)
        _tickets[key] = t
    return t


class Stats:
    """Per-channel statistics for the BN apply kernels: ``parts == 1`` -> ``buf`` is the finished
    [2][C] result; ``parts > 1`` -> ``buf`` holds [parts][3][C] level-1 partials that the
    consuming kernel merges in its prologue (norm.hip read_stats). Used as a tensor (tests,
    inspection) it materialises the finished [2][C] statistics (``final()``, torch ops: off the
    training hot path)."""
    __slots__ = ("buf", "parts", "mode", "_final")

    def __init__(self, buf, parts, mode=0):
        self.buf, self.parts, self.mode, self._final = buf, int(parts), int(mode), None

    def final(self):
        if self.parts == 1:
            return self.buf
        if self._final is None:
            p = self.buf.double()
            C = p.shape[2]
            parts = self.parts
            if self.mode == 0:  # Chan merges in part order (as read_stats)
                n, mean, m2 = p[0, 0].clone(), p[0, 1].clone(), p[0, 2].clone()
                for k in range(1, parts):
                    nb, mb, m2b = p[k, 0], p[k, 1], p[k, 2]
                    tot = n + nb
                    d = mb - mean
                    safe = torch.where(tot > 0, tot, torch.ones_like(tot))
                    mean = torch.where(tot > 0, mean + d * nb / safe, mean)
                    m2 = m2 + m2b + d * d * n * nb / safe
                    n = tot
                var = torch.where(n > 0, m2 / torch.where(n > 0, n, torch.ones_like(n)), torch.zeros_like(n))
                out = torch.cat([mean, var])
            else:
                out = torch.cat([p[:, 0].sum(0), p[:, 1].sum(0)])
            self._final = out.float().reshape(2 * C)
        return self._final

    def __getattr__(self, k):
        return getattr(self.final(), k)

    def __getitem__(self, i):
        return self.final()[i]


def prewarm_tickets(device, slots=("loss",)):
    """Create the calling stream's ticket words now (call it on a graph's capture stream before the
    capture): created during a capture, their zeroing would be re-run by every replay."""
    for s in slots:
        _ticket(torch.device(device), 0, slot=s)


def stat_reduce(mode, slab, rows, C, out):
    """Deterministic slab reduce (norm.hip bn_stat_reduce): mode 0 = Welford (count, mean, M2)
    tile triples -> (mean, biased var); mode 1 = (sum a, sum b) rows -> sums. Returns
    :class:`Stats` (``out`` when one block covered all rows, else the partials buffer).
    (Handing small slabs to the consumers raw instead measured no faster: the consumer prologue's
    merge costs what the launch saves, `profiles/experiment_raw_stats_r4.md`.)"""
    K = kernels()
    ny = K.bn_stat_parts(rows)
    part = _empty((ny, 3, C), F32, slab.device) if ny > 1 else None
    K.bn_stat_reduce(mode, slab.data_ptr(), rows, C, out.data_ptr(), ptr(part), 0, stream_ptr())
    return Stats(part if ny > 1 else out, ny, mode)


def _stats(s):
    """(pointer, parts) of a Stats / plain finished [2][C] tensor / None."""
    if s is None:
        return 0, 1
    if isinstance(s, Stats):
        return s.buf.data_ptr(), s.parts
    return s.data_ptr(), 1


_TRACE_PARTIAL = os.environ.get("DCNN_TRACE_PARTIAL", "0") == "1"
_traced_partial = set()


def _trace_partial(kind, x):
    """DCNN_TRACE_PARTIAL=1: report (once per call site and shape) every standalone BatchNorm
    statistics pass, i.e. a BatchNorm whose producer / consumer kernel could not emit its sums."""
    if not _TRACE_PARTIAL:
        return
    import sys
    import traceback
    fr = [f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in traceback.extract_stack(limit=8)[:-2]]
    key = (kind, tuple(x.shape), tuple(fr))
    if key not in _traced_partial:
        _traced_partial.add(key)
        print(f"[bn_partial] {kind} {tuple(x.shape)} <- {' <- '.join(reversed(fr))}", file=sys.stderr)


def bn_stats_raw(x, partial=None):
    """The (slab, rows, sums) statistics rows of x before the reduce (the producing conv's
    epilogue slab, else a bn_partial pass)."""
    if partial is not None:
        return partial
    K = kernels()
    R, C = _rc(x)
    rows = K.bn_partial_rows(R, C)
    slab = _empty((rows, 3, C), F32, x.device)
    sums = _empty((2 * C,), F32, x.device)
    _trace_partial("fwd", x)
    K.bn_partial(dt_code(x.dtype), x.data_ptr(), 0, 0, 0, 0, 0, R, C, slab.data_ptr(), 0, 0, stream_ptr())
    return slab, rows, sums


def bn_bwd_stats_raw(dy, x, mean, istd):
    """Backward statistics rows (sum dy, sum dy * xhat) of x before the reduce: (slab, rows, sums)."""
    K = kernels()
    R, C = _rc(x)
    rows = K.bn_partial_rows(R, C)
    slab = _empty((rows, 2, C), F32, x.device)
    sums = _empty((2 * C,), F32, x.device)
    _trace_partial("bwd_raw", x)
    K.bn_partial(dt_code(x.dtype), x.data_ptr(), dy.data_ptr(), 0, 0, mean.data_ptr(), istd.data_ptr(), R, C,
                 slab.data_ptr(), 1, 0, stream_ptr())
    return slab, rows, sums


def bn_bwd_apply_dual(dy, a, b):
    """Data gradients of two training BatchNorms fed the same (masked) gradient ``dy`` in one pass
    (norm.hip bn_bwd_apply_dual); ``a``/``b`` = (layer, its forward cache entry (x, _, mean, istd,
    _), reduced backward :class:`Stats`). Accumulates each layer's dgamma / dbeta."""
    R, C = _rc(dy)
    outs, sides = [], []
    for layer, ent, st in (a, b):
        x, _, mean, istd, _ = ent
        dx = _empty(x.shape, x.dtype, x.device, True)
        sp, parts = _stats(st)
        dg = layer._grads[0].view(-1) if layer.affine else None
        db = layer._grads[1].view(-1) if layer.affine else None
        sides.append((x.data_ptr(), dx.data_ptr(), mean.data_ptr(), istd.data_ptr(), ptr(layer._gamma()), sp, parts,
                      float(R), ptr(dg), ptr(db)))
        outs.append(dx)
    if not kernels().bn_bwd_apply_dual(dy.data_ptr(), sides[0], sides[1], R, C, stream_ptr()):
        raise RuntimeError("bn_bwd_apply_dual: unsupported shape")
    return outs[0], outs[1]


def stat_reduce_pair(mode, a, b, C):
    """Two independent forward/backward statistics reduces of the same C in ONE launch
    (norm.hip bn_stat_reduce2); ``a``/``b`` = (slab, rows, out). Returns two :class:`Stats`."""
    K = kernels()
    res, ptrs = [], []
    for slab, rows, out in (a, b):
        ny = K.bn_stat_parts(rows)
        part = _empty((ny, 3, C), F32, slab.device) if ny > 1 else None
        ptrs.append((slab.data_ptr(), rows, out.data_ptr(), ptr(part)))
        res.append(Stats(part if ny > 1 else out, ny, mode))
    (s1, r1, o1, p1), (s2, r2, o2, p2) = ptrs
    K.bn_stat_reduce2(mode, s1, r1, o1, p1, s2, r2, o2, p2, C, stream_ptr())
    return res[0], res[1]


def bn_stats(x, partial=None):
    """Per-channel (mean, biased variance) of x (NHWC), as one [2][C] fp32 tensor. Uses the
    producing conv's epilogue Welford slab if given, else a bn_partial pass; the reduction is
    deterministic and cancellation-free (Chan merges of pivot-shifted tile statistics)."""
    K = kernels()
    R, C = _rc(x)
    st = stream_ptr()
    if partial is None:
        rows = K.bn_partial_rows(R, C)
        slab = _empty((rows, 3, C), F32, x.device)
        sums = _empty((2 * C,), F32, x.device)
        _trace_partial("fwd", x)
        K.bn_partial(dt_code(x.dtype), x.data_ptr(), 0, 0, 0, 0, 0, R, C, slab.data_ptr(), 0, 0, st)
    else:
        slab, rows, sums = partial
    return stat_reduce(0, slab, rows, C, sums)


def bn_apply(x, sums, count, gamma, beta, eps, *, residual=None, relu=False, save=None, running=None,
             momentum=0.1, use_running=False):
    R, C = _rc(x)
    y = _empty(x.shape, x.dtype, x.device, True)
    sm, si = save if save is not None else (None, None)
    rm, rv = running if running is not None else (None, None)
    sp, parts = _stats(sums)
    kernels().bn_apply(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), R, C, sp, parts, float(count), ptr(gamma),
                       ptr(beta), float(eps), ptr(residual), int(relu), ptr(sm), ptr(si), ptr(rm), ptr(rv),
                       float(momentum), int(use_running), stream_ptr())
    return y


class BnDeferred:
    """A BatchNorm whose apply is deferred into the consumer (a residual block's tail BatchNorm
    applies its projection shortcut's BatchNorm on the fly: :func:`bn_apply_dual`)."""
    __slots__ = ("x", "sums", "count", "gamma", "beta", "eps", "save", "running", "momentum", "use_running")

    def __init__(self, x, sums, count, gamma, beta, eps, save, running, momentum, use_running):
        self.x, self.sums, self.count, self.gamma, self.beta, self.eps = x, sums, count, gamma, beta, eps
        self.save, self.running, self.momentum, self.use_running = save, running, momentum, use_running

    def reduced(self):
        """Reduce raw statistics rows (left raw so a consumer can pair the reduce with its own)."""
        if isinstance(self.sums, tuple):
            slab, rows, out = self.sums
            self.sums = stat_reduce(0, slab, rows, out.numel() // 2, out)
        return self

    def side(self):
        self.reduced()
        sp, parts = _stats(self.sums)
        sm, si = self.save if self.save is not None else (None, None)
        rm, rv = self.running if self.running is not None else (None, None)
        return (self.x.data_ptr(), sp, parts, float(self.count), ptr(self.gamma), ptr(self.beta), float(self.eps),
                ptr(sm), ptr(si), ptr(rm), ptr(rv), float(self.momentum), int(self.use_running))

    def materialize(self):
        """The deferred BatchNorm's output as a tensor (when the consumer cannot fuse it)."""
        self.reduced()
        return bn_apply(self.x, self.sums, self.count, self.gamma, self.beta, self.eps, save=self.save,
                        running=self.running, momentum=self.momentum, use_running=self.use_running)




def bn_dual_ok(x):
    return _BN_DUAL and x.dtype == BF16 and bool(kernels().bn_apply_dual_supported(*_rc(x)))


def bn_apply_dual(x, sums, count, gamma, beta, eps, other: BnDeferred, *, relu=False, save=None, running=None,
                  momentum=0.1, use_running=False):
    """act(bn(x) + other's BatchNorm output) in one pass (norm.hip bn_apply_dual)."""
    R, C = _rc(x)
    assert tuple(other.x.shape) == tuple(x.shape) and other.x.dtype == x.dtype == BF16
    y = _empty(x.shape, x.dtype, x.device, True)
    me = BnDeferred(x, sums, count, gamma, beta, eps, save, running, momentum, use_running)
    if not kernels().bn_apply_dual(me.side(), other.side(), y.data_ptr(), R, C, int(relu), stream_ptr()):
        raise RuntimeError("bn_apply_dual: unsupported shape")
    return y


def bn_relu_maxpool_ok(x, ph, pw, sh, sw, pdh, pdw):
    """Can :func:`bn_relu_maxpool` take this BatchNorm+ReLU+max-pool? Its backward relies on the
    fused max-pool backward (:func:`maxpool_bwd` with ``bnb``), so both must be available."""
    if not _BNB or x.dtype != BF16 or not x.is_contiguous(memory_format=CL):
        return False
    N, C, H, W = x.shape
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    g = (N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw)
    K = kernels()
    return K.bn_relu_maxpool_supported(*g) and K.maxpool_bwd_bnb_supported(*g)


def bn_relu_maxpool(x, sums, count, gamma, beta, eps, pool, *, save, running, momentum=0.1):
    """Training BatchNorm (batch statistics ``sums``) + ReLU + max-pool ``pool`` = (ph, pw, sh, sw,
    pdh, pdw) in one pass: returns the pooled output and the window argmax (max-pool layout)."""
    N, C, H, W = x.shape
    ph, pw, sh, sw, pdh, pdw = pool
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    y = _empty((N, C, OH, OW), BF16, x.device, True)
    idx = _empty((N, OH, OW, C), torch.uint8, x.device)
    sm, si = save
    rm, rv = running
    sp, parts = _stats(sums)
    kernels().bn_relu_maxpool(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw,
                              sp, parts, float(count), ptr(gamma), ptr(beta), float(eps), sm.data_ptr(),
                              si.data_ptr(), ptr(rm), ptr(rv), float(momentum), stream_ptr())
    return y, idx


def bn_backward(dy, x, yout, mean, istd, gamma, dgamma, dbeta, *, want_masked=False, eval_mode=False, fused=None):
    """Returns (dx, masked_dy|None). yout given => ReLU was fused: dy' = dy * (yout > 0).

    ``fused`` = (slab, rows, sums) when the producer of ``dy`` already applied the ReLU mask and
    wrote the backward statistics in its epilogue (:class:`BnbRequest`): only the slab reduce
    and the apply pass remain.
    """
    K = kernels()
    R, C = _rc(x)
    st = stream_ptr()
    dt = dt_code(x.dtype)
    if fused is not None and not eval_mode:
        slab, rows, sums = fused
        sp, parts = _stats(stat_reduce(1, slab, rows, C, sums))
        dx = _empty(x.shape, x.dtype, x.device, True)
        K.bn_bwd_apply(dt, dy.data_ptr(), 0, x.data_ptr(), dx.data_ptr(), R, C, mean.data_ptr(), istd.data_ptr(),
                       ptr(gamma), sp, parts, float(R), ptr(dgamma), ptr(dbeta), 0, st)
        return dx, (dy if want_masked else None)
    dmask = _empty(dy.shape, dy.dtype, dy.device, True) if (want_masked and yout is not None) else None
    sums = None
    # the (sum dy', sum dy' * xhat) pass: the batch-statistics backward needs it, and so does a
    # frozen-statistics (eval-mode) backward that still accumulates the affine gradients or
    # returns the masked gradient (bn_bwd_apply adds the sums to dgamma / dbeta either way and
    # uses them for dx only in training mode)
    if not eval_mode or dgamma is not None or dbeta is not None or dmask is not None:
        rows = K.bn_partial_rows(R, C)
        slab = _empty((rows, 2, C), F32, x.device)
        sums = _empty((2 * C,), F32, x.device)
        _trace_partial("bwd", x)
        K.bn_partial(dt, x.data_ptr(), dy.data_ptr(), ptr(yout), ptr(dmask), mean.data_ptr(), istd.data_ptr(), R, C,
                     slab.data_ptr(), 1, 0, st)
        sums = stat_reduce(1, slab, rows, C, sums)
    dx = _empty(x.shape, x.dtype, x.device, True)
    src = dmask if dmask is not None else dy
    sp, parts = _stats(sums)
    K.bn_bwd_apply(dt, src.data_ptr(), 0 if dmask is not None else ptr(yout), x.data_ptr(), dx.data_ptr(), R, C,
                   mean.data_ptr(), istd.data_ptr(), ptr(gamma), sp, parts, float(R), ptr(dgamma), ptr(dbeta),
                   int(eval_mode), st)
    return dx, dmask


def gn_fwd(x, groups, gamma, beta, eps):
    N, C, H, W = x.shape
    y = _empty(x.shape, x.dtype, x.device, True)
    mean = _empty((N * groups,), F32, x.device)
    istd = _empty_like(mean)
    kernels().gn_fwd(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), N, H * W, C, groups, ptr(gamma), ptr(beta),
                     float(eps), mean.data_ptr(), istd.data_ptr(), stream_ptr())
    return y, mean, istd


def gn_bwd(dy, x, groups, gamma, mean, istd, dgamma, dbeta):
    N, C, H, W = x.shape
    dx = _empty(x.shape, x.dtype, x.device, True)
    aff = _empty((N, 2, C), F32, x.device)  # per-image affine partials
    kernels().gn_bwd(dt_code(x.dtype), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), N, H * W, C, groups, ptr(gamma),
                     mean.data_ptr(), istd.data_ptr(), ptr(dgamma), ptr(dbeta), aff.data_ptr(), stream_ptr())
    return dx


# ------------------------------------------------------------------------------ pooling
def pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw):
    return (H + 2 * pdh - ph) // sh + 1, (W + 2 * pdw - pw) // sw + 1


def maxpool_fwd(x, ph, pw, sh, sw, pdh, pdw):
    _check_act(x, "maxpool")
    N, C, H, W = x.shape
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    y = _empty((N, C, OH, OW), x.dtype, x.device, True)
    idx = _empty((N, OH, OW, C), torch.uint8, x.device)
    assert ph * pw <= 256
    kernels().maxpool_fwd(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW, ph, pw,
                          sh, sw, pdh, pdw, stream_ptr())
    return y, idx


def maxpool_bwd(dy, idx, x_shape, ph, pw, sh, sw, pdh, pdw, *, ypool=None, bnb=None):
    """Gather-form max-pool backward. With ``bnb`` (the BatchNorm+ReLU that produced the pool's
    input, see :class:`BnbRequest`) and the pool output ``ypool``, the ReLU mask (pooled value > 0)
    and that BatchNorm's backward statistics are fused in (``dx._bnb`` attached)."""
    N, C, H, W = x_shape
    OH, OW = dy.shape[2], dy.shape[3]
    K = kernels()
    dx = _empty((N, C, H, W), dy.dtype, dy.device, True)
    g = (N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw)
    # the kernel masks with (pooled value > 0): only valid when a ReLU sits between BN and pool
    if (bnb is not None and _BNB and (bnb.y is not None or bnb.pooled) and ypool is not None and dy.dtype == BF16 and bnb.x.dtype == BF16
            and tuple(bnb.x.shape) == (N, C, H, W) and bnb.x.is_contiguous(memory_format=CL)
            and K.maxpool_bwd_bnb_supported(*g)):
        rows = K.maxpool_bwd_bnb_rows(*g)
        slab = _empty((rows, 2, C), F32, dy.device)
        sums = _empty((2 * C,), F32, dy.device)  # zeroed in-kernel
        K.maxpool_bwd_bnb(dy.data_ptr(), idx.data_ptr(), ypool.data_ptr(), bnb.x.data_ptr(), bnb.mean.data_ptr(),
                          bnb.istd.data_ptr(), dx.data_ptr(), *g, slab.data_ptr(), sums.data_ptr(), stream_ptr())
        dx._bnb = (bnb.bn, slab, rows, sums)
        return dx
    K.maxpool_bwd(dt_code(dy.dtype), dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), *g, stream_ptr())
    return dx


def avgpool_fwd(x, ph, pw, sh, sw, pdh, pdw):
    _check_act(x, "avgpool")
    N, C, H, W = x.shape
    OH, OW = pool_out_hw(H, W, ph, pw, sh, sw, pdh, pdw)
    y = _empty((N, C, OH, OW), x.dtype, x.device, True)
    kernels().avgpool_fwd(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), N, H, W, C, OH, OW, ph, pw, sh, sw, pdh, pdw,
                          stream_ptr())
    return y


def avgpool_bwd(dy, x_shape, ph, pw, sh, sw, pdh, pdw):
    N, C, H, W = x_shape
    OH, OW = dy.shape[2], dy.shape[3]
    dy = dy.contiguous(memory_format=CL)
    dx = _empty((N, C, H, W), dy.dtype, dy.device, True)
    kernels().avgpool_bwd(dt_code(dy.dtype), dy.data_ptr(), dx.data_ptr(), N, H, W, C, OH, OW, ph, pw, sh, sw, pdh,
                          pdw, stream_ptr())
    return dx


# ------------------------------------------------------------------------------ activations
ACT_CODES = {"relu": 0, "leaky_relu": 1, "elu": 2, "sigmoid": 3, "tanh": 4, "linear": 5}


def act_fwd(x, kind, alpha=0.01):
    y = _empty_like(x)
    kernels().act_fwd(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), x.numel(), ACT_CODES[kind], float(alpha),
                      stream_ptr())
    return y


def act_bwd(x, dy, kind, alpha=0.01):
    dy = dy.contiguous(memory_format=CL) if x.dim() == 4 and x.is_contiguous(memory_format=CL) else dy.contiguous()
    dx = _empty_like(x)
    kernels().act_bwd(dt_code(x.dtype), x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), ACT_CODES[kind],
                      float(alpha), stream_ptr())
    return dx


def softmax_channels(x):
    """softmax over dim 1 of an NCHW-logical / NHWC-physical tensor (channel innermost)."""
    N, C = x.shape[0], x.shape[1]
    rows = x.numel() // C
    y = _empty_like(x)
    kernels().softmax_rows(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), rows, C, stream_ptr())
    return y


def softmax_channels_bwd(y, dy):
    C = y.shape[1]
    rows = y.numel() // C
    dy = dy.contiguous(memory_format=CL) if y.dim() == 4 else dy.contiguous()
    dx = _empty_like(y)
    kernels().softmax_rows_bwd(dt_code(y.dtype), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), rows, C, stream_ptr())
    return dx


def dropout(x, p, seed, slot=None):
    """Inverted dropout with a Philox mask of (seed, *slot). ``slot``: a 1-element int64 device
    tensor written by :func:`counter_bump` (graph-replay safe: the draw index lives on the device)."""
    y = _empty_like(x)
    kernels().dropout(dt_code(x.dtype), x.data_ptr(), y.data_ptr(), x.numel(), float(p), int(seed) & ((1 << 64) - 1),
                      ptr(slot), stream_ptr())
    return y


def counter_bump(ctr, slot):
    """slot = ++ctr on the device (both 1-element int64 tensors)."""
    kernels().counter_bump(ctr.data_ptr(), slot.data_ptr(), stream_ptr())


# ------------------------------------------------------------------------------ loss / optim
LOSS_CODES = {"crossentropy": 0, "softmax_crossentropy": 1, "logsoftmax_crossentropy": 2, "mse": 3, "mae": 4,
              "huber": 5}


def loss_fused(pred2d, target2d=None, labels=None, kind="softmax_crossentropy", param=1e-15, want_grad=True,
               grad_scale=1.0):
    """Returns (loss[1] f32 device, grad|None, correct[1] int32 device). No host sync. The gradient
    is additionally multiplied by ``grad_scale`` inside the kernel (data parallel: 1 / world)."""
    N, C = pred2d.shape
    pred2d = pred2d.contiguous()
    grad = _empty_like(pred2d) if want_grad else None
    loss = torch.empty((1,), dtype=F32, device=pred2d.device)
    correct = torch.empty((1,), dtype=torch.int32, device=pred2d.device)
    tgt = None
    if target2d is not None:
        tgt = target2d.reshape(N, C).to(F32).contiguous()
    lab = labels.to(torch.int64).contiguous() if labels is not None else None
    K = kernels()
    ws = _empty((K.loss_workspace_floats(N),), F32, pred2d.device) if N > 4 else None
    tk = _ticket(pred2d.device, 0, slot="loss") if N > 4 else None
    K.loss_fused(dt_code(pred2d.dtype), pred2d.data_ptr(), ptr(tgt), ptr(lab), ptr(grad), loss.data_ptr(),
                 correct.data_ptr(), N, C, LOSS_CODES[kind], float(param), float(grad_scale), ptr(ws), ptr(tk),
                 stream_ptr())
    return loss, grad, correct


def adam_step(p, g, m, v, shadow, lr, b1, b2, eps, bc1, bc2, wd, decoupled, hyper=None):
    kernels().adam_step(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), ptr(shadow), p.numel(), float(lr),
                        float(b1), float(b2), float(eps), float(bc1), float(bc2), float(wd), int(decoupled),
                        ptr(hyper), stream_ptr())


def sgd_step(p, g, vel, shadow, lr, momentum, hyper=None):
    kernels().sgd_step(p.data_ptr(), g.data_ptr(), ptr(vel), ptr(shadow), p.numel(), float(lr), float(momentum),
                       ptr(hyper), stream_ptr())


def zero_(t):
    """Zero a dense GPU tensor on the current stream with the library's own fill kernel (no ATen
    fill on the hot path). Not hipMemsetAsync: captured into a hipGraph, a memset node wrote
    garbage from its second replay on (ROCm 7.2; observed with a capture of two memset nodes)."""
    assert t.is_cuda and (t.is_contiguous() or t.is_contiguous(memory_format=CL))
    kernels().zero_bytes(t.data_ptr(), t.numel() * t.element_size(), stream_ptr(t.device))
    return t


def cast_bf16(src, dst):
    kernels().cast_f32_bf16(src.data_ptr(), dst.data_ptr(), src.numel(), stream_ptr())


class WeightTransposer:
    """Regenerates every conv's dgrad operand ([Ci][KH][KW][Co] bf16) from the bf16 shadow
    weights in ONE kernel launch per step (instead of one launch per conv)."""

    def __init__(self, convs):
        self.convs = [c for c in convs if c.in_channels % 8 == 0 and c.out_channels % 8 == 0]
        rows = []
        self.max_tiles = 0  # 64x64 (co, ci) tiles per tap: the launch's x extent
        for c in self.convs:
            w = c.weight_operand(0)
            Co, Ci, KH, KW = w.shape
            c._wt_buf = _arena.persistent((Ci, KH, KW, Co), BF16, w.device)
            rows.append([w.data_ptr(), c._wt_buf.data_ptr(), Co, KH * KW, Ci])
            self.max_tiles = max(self.max_tiles, KH * KW * ((Co + 63) // 64) * ((Ci + 63) // 64))
        self.table = torch.tensor(rows, dtype=torch.int64).to(self.convs[0]._wt_buf.device) if rows else None

    def run(self):
        if self.table is None:
            return
        kernels().multi_weight_transpose(self.table.data_ptr(), len(self.convs), self.max_tiles, stream_ptr())
        for c in self.convs:
            c._wt_valid = True

    def invalidate(self):
        for c in self.convs:
            c._wt_valid = False


def im2col(x, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x.shape
    OH, OW = conv_out_hw(H, W, kh, kw, sh, sw, ph, pw)
    x = x.contiguous().float()
    col = _empty((C * kh * kw, N * OH * OW), F32, x.device)
    kernels().im2col(x.data_ptr(), col.data_ptr(), N, C, H, W, kh, kw, sh, sw, ph, pw, OH, OW, stream_ptr())
    return col


def col2im(col, x_shape, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x_shape
    OH, OW = conv_out_hw(H, W, kh, kw, sh, sw, ph, pw)
    x = _empty((N, C, H, W), F32, col.device)
    kernels().col2im(col.contiguous().data_ptr(), x.data_ptr(), N, C, H, W, kh, kw, sh, sw, ph, pw, OH, OW,
                     stream_ptr())
    return x
