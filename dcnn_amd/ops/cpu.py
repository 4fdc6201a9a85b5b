"""Native CPU backend (``_native.cpu``, csrc/native/cpu_ops.cpp + cpu_gemm.cpp).

The CPU counterpart of ``ops/hip.py``: every layer's CPU path runs these C++ kernels (blocked
AVX2 GEMM, per-sample im2col convolution, two-pass BatchNorm statistics, pooling with argmax
indices, fused losses, flat-buffer optimizers) on the native thread pool, in float32 or float64,
NCHW contiguous. ATen is only the test oracle (tests/test_cpu_backend.py).

Reference: src/ops/cpu/skernels.cpp / dkernels.cpp, src/math/cpu/sgemm.cpp / dgemm.cpp,
include/tensor/cpu/tensor_ops.hpp:283, src/nn/layers_impl/cpu/*_ops.cpp.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._ext import native

_DT = {torch.float32: 0, torch.float64: 1}
ACT_CODES = {"linear": 0, "relu": 1, "leaky_relu": 2, "elu": 3, "sigmoid": 4, "tanh": 5}
LOSS_CODES = {"crossentropy": 0, "softmax_crossentropy": 1, "logsoftmax_crossentropy": 1, "mse": 2, "mae": 3,
              "huber": 4}


def C():
    return native().cpu


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"CPU backend computes in float32 / float64, got {t.dtype}") from None


def p(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.is_cuda:
        raise TypeError("CPU backend got a GPU tensor")
    return t if t.is_contiguous() else t.contiguous()


def _same(ref: torch.Tensor, *ts):
    for t in ts:
        if t is not None and t.dtype != ref.dtype:
            raise TypeError(f"dtype mismatch: {t.dtype} vs {ref.dtype}")


def set_num_threads(n: int) -> None:
    C().set_num_threads(int(n))


def get_num_threads() -> int:
    return int(C().get_num_threads())


# ------------------------------------------------------------------ GEMM
def gemm(a: torch.Tensor, b: torch.Tensor, ta: bool = False, tb: bool = False, alpha: float = 1.0,
         beta: float = 0.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = alpha * op(a) @ op(b) + beta * out for 2-D row-major tensors."""
    a, b = _c(a), _c(b)
    _same(a, b)
    M, K = (a.shape[1], a.shape[0]) if ta else (a.shape[0], a.shape[1])
    K2, N = (b.shape[1], b.shape[0]) if tb else (b.shape[0], b.shape[1])
    if K != K2:
        raise ValueError(f"gemm: inner dims {K} vs {K2}")
    if out is None:
        out = torch.empty((M, N), dtype=a.dtype)
        beta = 0.0
    elif tuple(out.shape) != (M, N) or not out.is_contiguous():
        raise ValueError("gemm: out must be a contiguous [M, N] tensor")
    C().gemm(dt(a), ta, tb, M, N, K, float(alpha), a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1], float(beta),
             out.data_ptr(), N)
    return out


# ------------------------------------------------------------------ generic elementwise / reduce
def elementwise(mode: int, op: int, a, b=None, out=None, s0=0.0, s1=0.0):
    a = _c(a)
    b = _c(b)
    _same(a, b)
    if b is not None and b.numel() != a.numel():
        raise ValueError("size mismatch")
    if out is None:
        out = torch.empty_like(a)
    C().elementwise(dt(a), mode, op, a.data_ptr(), p(b), out.data_ptr(), a.numel(), float(s0), float(s1))
    return out


def ternary(op: int, a, b, c):
    a, b = _c(a), _c(b)
    _same(a, b, c)
    if not c.is_contiguous():
        raise ValueError("in-place target must be contiguous")
    C().elementwise(dt(a), 3, op, a.data_ptr(), b.data_ptr(), c.data_ptr(), a.numel(), 0.0, 0.0)
    return c


def axpy(alpha, x, y):
    x = _c(x)
    _same(x, y)
    C().elementwise(dt(x), 4, 0, x.data_ptr(), 0, y.data_ptr(), x.numel(), float(alpha), 0.0)
    return y


def reduce(op: int, a, b=None) -> torch.Tensor:
    a, b = _c(a), _c(b)
    v = C().reduce(dt(a), op, a.data_ptr(), p(b), a.numel())
    return torch.tensor([v], dtype=a.dtype)


def fill_random(a: torch.Tensor, lo: float, hi: float, seed: int, normal: bool) -> torch.Tensor:
    if not a.is_contiguous():
        raise ValueError("fill target must be contiguous")
    C().fill_random(dt(a), a.data_ptr(), a.numel(), int(seed) & ((1 << 64) - 1), float(lo), float(hi), int(normal))
    return a


def transpose_2d(a, rows, cols, batch=1):
    a = _c(a)
    out = torch.empty(batch * rows * cols, dtype=a.dtype)
    C().transpose2d(dt(a), a.data_ptr(), out.data_ptr(), batch, rows, cols)
    return out.view(batch, cols, rows) if batch > 1 else out.view(cols, rows)


def swap01(a: torch.Tensor) -> torch.Tensor:
    """[A][B][H][W] -> [B][A][H][W] (NCHW <-> CNHW)."""
    a = _c(a)
    A, B, H, W = a.shape
    out = torch.empty((B, A, H, W), dtype=a.dtype)
    C().swap01(dt(a), a.data_ptr(), out.data_ptr(), A, B, H * W)
    return out


def pad2d(x, ph, pw, value=0.0):
    x = _c(x)
    N, Cc, H, W = x.shape
    y = torch.empty((N, Cc, H + 2 * ph, W + 2 * pw), dtype=x.dtype)
    C().pad2d(dt(x), x.data_ptr(), y.data_ptr(), N * Cc, H, W, ph, pw, float(value))
    return y


def crop2d(x, top, left, oh, ow):
    x = _c(x)
    N, Cc, H, W = x.shape
    if top < 0 or left < 0 or top + oh > H or left + ow > W:
        raise ValueError("crop window outside the input")
    y = torch.empty((N, Cc, oh, ow), dtype=x.dtype)
    C().crop2d(dt(x), x.data_ptr(), y.data_ptr(), N * Cc, H, W, top, left, oh, ow)
    return y


def _odim(i, k, s, pd):
    return (i + 2 * pd - k) // s + 1


def im2col(x, kh, kw, sh, sw, ph, pw):
    """[C*KH*KW, N*OH*OW] column matrix (the reference layout)."""
    x = _c(x)
    N, Cc, H, W = x.shape
    OH, OW = _odim(H, kh, sh, ph), _odim(W, kw, sw, pw)
    col = torch.empty((Cc * kh * kw, N * OH * OW), dtype=x.dtype)
    C().im2col(dt(x), x.data_ptr(), col.data_ptr(), N, Cc, H, W, kh, kw, sh, sw, ph, pw)
    return col


def col2im(col, shape, kh, kw, sh, sw, ph, pw):
    col = _c(col)
    N, Cc, H, W = shape
    x = torch.empty((N, Cc, H, W), dtype=col.dtype)
    C().col2im(dt(col), col.data_ptr(), x.data_ptr(), N, Cc, H, W, kh, kw, sh, sw, ph, pw)
    return x


# ------------------------------------------------------------------ layers
def conv2d_fwd(x, w, bias, stride, pad):
    x, w, bias = _c(x), _c(w), _c(bias)
    _same(x, w, bias)
    N, Ci, H, W = x.shape
    Co, Ci2, KH, KW = w.shape
    if Ci != Ci2:
        raise ValueError(f"conv2d: {Ci} input channels, weights expect {Ci2}")
    OH, OW = _odim(H, KH, stride[0], pad[0]), _odim(W, KW, stride[1], pad[1])
    y = torch.empty((N, Co, OH, OW), dtype=x.dtype)
    C().conv2d_fwd(dt(x), x.data_ptr(), w.data_ptr(), p(bias), y.data_ptr(), N, Ci, H, W, Co, KH, KW, stride[0],
                   stride[1], pad[0], pad[1])
    return y


def conv2d_bwd(x, w, dy, stride, pad, grad_w, grad_b=None, need_dx=True):
    """grad_w (+)= dW, grad_b (+)= sum(dy); returns dx (or None). grad_w/grad_b must be contiguous."""
    x, w, dy = _c(x), _c(w), _c(dy)
    _same(x, w, dy, grad_w, grad_b)
    N, Ci, H, W = x.shape
    Co, _, KH, KW = w.shape
    for g in (grad_w, grad_b):
        if g is not None and not g.is_contiguous():
            raise ValueError("gradient accumulators must be contiguous")
    dx = torch.empty_like(x) if need_dx else None
    C().conv2d_bwd(dt(x), x.data_ptr(), w.data_ptr(), dy.data_ptr(), p(dx), grad_w.data_ptr(), p(grad_b), N, Ci, H, W,
                   Co, KH, KW, stride[0], stride[1], pad[0], pad[1])
    return dx


def dense_fwd(x2d, w2d, bias):
    x2d, w2d, bias = _c(x2d), _c(w2d), _c(bias)
    _same(x2d, w2d, bias)
    N, In = x2d.shape
    Out = w2d.shape[0]
    y = torch.empty((N, Out), dtype=x2d.dtype)
    C().dense_fwd(dt(x2d), x2d.data_ptr(), w2d.data_ptr(), p(bias), y.data_ptr(), N, In, Out)
    return y


def dense_bwd(x2d, w2d, dy2d, grad_w, grad_b=None, need_dx=True):
    x2d, w2d, dy2d = _c(x2d), _c(w2d), _c(dy2d)
    _same(x2d, w2d, dy2d, grad_w, grad_b)
    N, In = x2d.shape
    Out = w2d.shape[0]
    dx = torch.empty_like(x2d) if need_dx else None
    C().dense_bwd(dt(x2d), x2d.data_ptr(), w2d.data_ptr(), dy2d.data_ptr(), p(dx), grad_w.data_ptr(), p(grad_b), N,
                  In, Out)
    return dx


def batchnorm_fwd(x, gamma, beta, eps, training, running_mean, running_var, momentum, relu=False, residual=None):
    """Returns (y, mean, istd). Training: batch statistics (two-pass), running stats updated with
    the unbiased variance; eval: running statistics."""
    x, residual = _c(x), _c(residual)
    _same(x, gamma, beta, residual, running_mean, running_var)
    N, Cc, H, W = x.shape
    y = torch.empty_like(x)
    mean = torch.empty(Cc, dtype=x.dtype)
    istd = torch.empty(Cc, dtype=x.dtype)
    C().batchnorm_fwd(dt(x), x.data_ptr(), y.data_ptr(), N, Cc, H * W, p(gamma), p(beta), float(eps), int(training),
                      p(running_mean), p(running_var), float(momentum), mean.data_ptr(), istd.data_ptr(), int(relu),
                      p(residual))
    return y, mean, istd


def batchnorm_bwd(x, dy, yout, mean, istd, gamma, dgamma, dbeta, training=True, want_masked=False, need_dx=True):
    """Returns (dx, masked_dy). ``yout`` given: dy is masked by (yout > 0) (fused ReLU)."""
    x, dy, yout = _c(x), _c(dy), _c(yout)
    _same(x, dy, yout, mean, istd, gamma, dgamma, dbeta)
    N, Cc, H, W = x.shape
    dx = torch.empty_like(x) if need_dx else None
    masked = torch.empty_like(dy) if want_masked else None
    C().batchnorm_bwd(dt(x), x.data_ptr(), dy.data_ptr(), p(yout), mean.data_ptr(), istd.data_ptr(), p(gamma), p(dx),
                      p(dgamma), p(dbeta), p(masked), N, Cc, H * W, int(training))
    return dx, masked


def groupnorm_fwd(x, G, gamma, beta, eps):
    x = _c(x)
    _same(x, gamma, beta)
    N, Cc, H, W = x.shape
    y = torch.empty_like(x)
    mean = torch.empty(N * G, dtype=x.dtype)
    istd = torch.empty(N * G, dtype=x.dtype)
    C().groupnorm_fwd(dt(x), x.data_ptr(), y.data_ptr(), N, Cc, H * W, G, p(gamma), p(beta), float(eps),
                      mean.data_ptr(), istd.data_ptr())
    return y, mean, istd


def groupnorm_bwd(x, dy, G, gamma, mean, istd, dgamma, dbeta):
    x, dy = _c(x), _c(dy)
    _same(x, dy, gamma, mean, istd, dgamma, dbeta)
    N, Cc, H, W = x.shape
    dx = torch.empty_like(x)
    C().groupnorm_bwd(dt(x), x.data_ptr(), dy.data_ptr(), mean.data_ptr(), istd.data_ptr(), p(gamma), dx.data_ptr(),
                      p(dgamma), p(dbeta), N, Cc, H * W, G)
    return dx


def maxpool_fwd(x, k, s, pd) -> Tuple[torch.Tensor, torch.Tensor]:
    x = _c(x)
    N, Cc, H, W = x.shape
    OH, OW = _odim(H, k[0], s[0], pd[0]), _odim(W, k[1], s[1], pd[1])
    y = torch.empty((N, Cc, OH, OW), dtype=x.dtype)
    idx = torch.empty((N, Cc, OH, OW), dtype=torch.int32)
    C().maxpool_fwd(dt(x), x.data_ptr(), y.data_ptr(), idx.data_ptr(), N * Cc, H, W, k[0], k[1], s[0], s[1], pd[0],
                    pd[1])
    return y, idx


def maxpool_bwd(dy, idx, in_shape):
    dy, idx = _c(dy), _c(idx)
    N, Cc, H, W = in_shape
    dx = torch.empty((N, Cc, H, W), dtype=dy.dtype)
    C().maxpool_bwd(dt(dy), dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N * Cc, H, W, dy.shape[2], dy.shape[3])
    return dx


def avgpool_fwd(x, k, s, pd):
    x = _c(x)
    N, Cc, H, W = x.shape
    OH, OW = _odim(H, k[0], s[0], pd[0]), _odim(W, k[1], s[1], pd[1])
    y = torch.empty((N, Cc, OH, OW), dtype=x.dtype)
    C().avgpool_fwd(dt(x), x.data_ptr(), y.data_ptr(), N * Cc, H, W, k[0], k[1], s[0], s[1], pd[0], pd[1])
    return y


def avgpool_bwd(dy, in_shape, k, s, pd):
    dy = _c(dy)
    N, Cc, H, W = in_shape
    dx = torch.empty((N, Cc, H, W), dtype=dy.dtype)
    C().avgpool_bwd(dt(dy), dy.data_ptr(), dx.data_ptr(), N * Cc, H, W, k[0], k[1], s[0], s[1], pd[0], pd[1])
    return dx


def act_fwd(x, kind, alpha=0.0):
    x = _c(x)
    y = torch.empty_like(x)
    C().act_fwd(dt(x), ACT_CODES[kind], x.data_ptr(), y.data_ptr(), x.numel(), float(alpha))
    return y


def act_bwd(x, dy, kind, alpha=0.0):
    x, dy = _c(x), _c(dy)
    _same(x, dy)
    dx = torch.empty_like(x)
    C().act_bwd(dt(x), ACT_CODES[kind], x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), float(alpha))
    return dx


def _nchw(x):
    N, Cc = x.shape[0], x.shape[1]
    return N, Cc, x.numel() // max(N * Cc, 1)


def softmax_channels(x):
    x = _c(x)
    y = torch.empty_like(x)
    C().softmax_channels(dt(x), x.data_ptr(), y.data_ptr(), *_nchw(x))
    return y


def softmax_channels_bwd(y, dy):
    y, dy = _c(y), _c(dy)
    dx = torch.empty_like(y)
    C().softmax_channels_bwd(dt(y), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), *_nchw(y))
    return dx


def loss_fused(pred2d, target2d=None, labels=None, kind="softmax_crossentropy", param=0.0, want_grad=True):
    """(loss[1], grad | None, correct[1] int32) — the CPU twin of ``hip.loss_fused``."""
    pred2d = _c(pred2d)
    N, Cn = pred2d.shape
    tgt = _c(target2d.to(pred2d.dtype)) if target2d is not None else None
    lab = _c(labels.to(torch.int64)) if labels is not None else None
    grad = torch.empty_like(pred2d) if want_grad else None
    l, cor = C().loss_fused(dt(pred2d), LOSS_CODES[kind], pred2d.data_ptr(), p(tgt), p(lab), p(grad), N, Cn,
                            float(param))
    return (torch.tensor([l], dtype=pred2d.dtype), grad, torch.tensor([cor], dtype=torch.int32))


def sgd_step(p_, g, vel, lr, momentum):
    C().sgd_step(dt(p_), p_.data_ptr(), g.data_ptr(), p(vel), p_.numel(), float(lr), float(momentum))


def adam_step(p_, g, m, v, lr, b1, b2, eps, bc1, bc2, wd, decoupled):
    C().adam_step(dt(p_), p_.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p_.numel(), float(lr), float(b1),
                  float(b2), float(eps), float(bc1), float(bc2), float(wd), int(decoupled))
