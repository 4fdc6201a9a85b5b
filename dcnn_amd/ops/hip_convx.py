"""Conv helpers outside the implicit-GEMM routing of ops/hip.py: the RGB stem kernels, weight layout
operands, and the explicit im2col + GEMM algorithm (``set_conv_algo("im2col")``; im2col.hip, the
reference's lowering src/nn/layers_impl/cuda/conv2d_ops.cu:78-98)."""
from __future__ import annotations

from ..runtime import arena as _arena
from ._ext import dt_code, kernels, ptr, stream_ptr
from .hip_base import (BF16, CL, F32, _NOBNB, _check_act, _empty, _nbytes, _rec, _reduce_wb,
                       conv_out_hw)


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
