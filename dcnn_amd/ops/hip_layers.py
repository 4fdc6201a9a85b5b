"""Dense layers, pooling, activations, loss, optimizer steps and layout helpers on the HIP kernels."""
from __future__ import annotations

import torch

from ..runtime import arena as _arena
from . import fusion
from ._ext import dt_code, kernels, ptr, stream_ptr
from .hip_base import (BF16, CL, F32, PLAIN, _NOBNB, _check_act, _empty, _empty_like, _g2_ok, _nbytes,
                       _reduce_wb, _ticket, conv_out_hw, pool_out_hw)


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


# ------------------------------------------------------------------------------ pooling
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
    if (bnb is not None and fusion.BNB and (bnb.y is not None or bnb.pooled) and ypool is not None and dy.dtype == BF16 and bnb.x.dtype == BF16
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
    """Regenerates every conv's dgrad operand ([Ci][KH][KW][Co]) from the bf16 shadow weights (or,
    on the fp32 compute path, the fp32 channels_last masters) in ONE kernel launch per step
    (instead of one launch per conv)."""

    def __init__(self, convs, dtype=BF16):
        self.dtype = dtype
        self.convs = [c for c in convs if c.in_channels % 8 == 0 and c.out_channels % 8 == 0]
        rows = []
        self.max_tiles = 0  # 64x64 (co, ci) tiles per tap: the launch's x extent
        for c in self.convs:
            w = c.weight_operand(0)
            Co, Ci, KH, KW = w.shape
            assert w.dtype == dtype and (w.is_contiguous(memory_format=CL) or KH * KW == 1)
            c._wt_buf = _arena.persistent((Ci, KH, KW, Co), dtype, w.device)
            rows.append([w.data_ptr(), c._wt_buf.data_ptr(), Co, KH * KW, Ci])
            self.max_tiles = max(self.max_tiles, KH * KW * ((Co + 63) // 64) * ((Ci + 63) // 64))
        self.table = torch.tensor(rows, dtype=torch.int64).to(self.convs[0]._wt_buf.device) if rows else None

    def run(self):
        if self.table is None:
            return
        kernels().multi_weight_transpose(self.table.data_ptr(), len(self.convs), self.max_tiles, stream_ptr(),
                                         int(self.dtype == F32))
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
