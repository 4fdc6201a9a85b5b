"""Device-agnostic generic ops (reference include/ops/ops.hpp:17-944).

Every op takes torch tensors and dispatches on their device: GPU tensors run the HIP kernels
of ``csrc/kernels/ops.hip`` (fp32; anything else raises — no silent fallback), CPU tensors run
the native C++ backend (``ops/cpu.py``, float32 and float64 — the reference's skernels.cpp /
dkernels.cpp pair) with the same op codes. Reductions return a 1-element *device* tensor
(the reference blocks and copies to the host on every call); call ``float()`` to
synchronise. The CPU random fills use the GPU's Philox-4x32-10 stream: the same seed gives the
same numbers on either device.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import cpu as _cpu
from ._ext import kernels, stream_ptr

_B = {"add": 0, "sub": 1, "mul": 2, "div": 3, "min": 4, "max": 5, "equal": 6, "greater": 7}
_U = {"sqrt": 16, "rsqrt": 17, "rcp": 18, "abs": 19, "neg": 20, "exp": 21, "log": 22, "copy": 23}
_T = {"fmadd": 32, "fmsub": 33, "fnmadd": 34}
CLAMP, SUB_MUL, MUL_ADD = 48, 49, 50


def _gpu(*ts) -> bool:
    on = [t.is_cuda for t in ts if t is not None]
    if any(on):
        for t in ts:
            if t is not None and (not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous()):
                raise TypeError("GPU generic ops take contiguous float32 CUDA tensors")
        return True
    return False


def _out(a, out):
    return torch.empty_like(a) if out is None else out


def _ew(mode, op, a, b=None, out=None, s0=0.0, s1=0.0):
    c = _out(a, out)
    if b is not None and b.numel() != a.numel():
        raise ValueError("size mismatch")
    kernels().elementwise(mode, op, a.data_ptr(), 0 if b is None else b.data_ptr(), c.data_ptr(), a.numel(),
                          float(s0), float(s1), stream_ptr())
    return c


# ---- binary
def _binary(name, torch_fn):
    def f(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if _gpu(a, b, out):
            return _ew(0, _B[name], a, b, out)
        return _cpu.elementwise(0, _B[name], a, b, out)
    f.__name__ = name
    return f


add = _binary("add", torch.add)
sub = _binary("sub", torch.sub)
mul = _binary("mul", torch.mul)
div = _binary("div", torch.div)
min = _binary("min", torch.minimum)  # noqa: A001
max = _binary("max", torch.maximum)  # noqa: A001
equal = _binary("equal", torch.eq)
greater = _binary("greater", torch.gt)


def _scalar(name, torch_fn):
    def f(a: torch.Tensor, s: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if _gpu(a, out):
            return _ew(1, _B[name], a, None, out, s)
        return _cpu.elementwise(1, _B[name], a, None, out, s)
    f.__name__ = name + "_scalar"
    return f


add_scalar = _scalar("add", torch.add)
sub_scalar = _scalar("sub", torch.sub)
mul_scalar = _scalar("mul", torch.mul)
div_scalar = _scalar("div", torch.div)
scalar_max = _scalar("max", lambda a, s: torch.clamp(a, min=s))


def _unary(name, torch_fn):
    def f(a: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if _gpu(a, out):
            return _ew(2, _U[name], a, None, out)
        return _cpu.elementwise(2, _U[name], a, None, out)
    f.__name__ = name
    return f


sqrt = _unary("sqrt", torch.sqrt)
rsqrt = _unary("rsqrt", torch.rsqrt)
rcp = _unary("rcp", torch.reciprocal)
abs = _unary("abs", torch.abs)  # noqa: A001
exp = _unary("exp", torch.exp)
log = _unary("log", torch.log)
copy = _unary("copy", torch.clone)


def clamp(a, lo, hi, out=None):
    if _gpu(a, out):
        return _ew(2, CLAMP, a, None, out, lo, hi)
    return _cpu.elementwise(2, CLAMP, a, None, out, lo, hi)


def sub_mul_scalar(a, sub_v, mul_v, out=None):
    """(a - sub_v) * mul_v"""
    if _gpu(a, out):
        return _ew(2, SUB_MUL, a, None, out, sub_v, mul_v)
    return _cpu.elementwise(2, SUB_MUL, a, None, out, sub_v, mul_v)


def mul_add_scalar(a, mul_v, add_v, out=None):
    """a * mul_v + add_v"""
    if _gpu(a, out):
        return _ew(2, MUL_ADD, a, None, out, mul_v, add_v)
    return _cpu.elementwise(2, MUL_ADD, a, None, out, mul_v, add_v)


def _ternary(name, torch_fn):
    def f(a, b, c):
        """In place on ``c``: fmadd c = a*b + c, fmsub c = a*b - c, fnmadd c = -(a*b) + c."""
        if _gpu(a, b, c):
            kernels().elementwise(3, _T[name], a.data_ptr(), b.data_ptr(), c.data_ptr(), a.numel(), 0.0, 0.0,
                                  stream_ptr())
            return c
        return _cpu.ternary(_T[name], a, b, c)
    f.__name__ = name
    return f


fmadd = _ternary("fmadd", lambda a, b, c: a * b + c)
fmsub = _ternary("fmsub", lambda a, b, c: a * b - c)
fnmadd = _ternary("fnmadd", lambda a, b, c: c - a * b)


def axpy(alpha: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """y += alpha * x (in place)."""
    if _gpu(x, y):
        kernels().elementwise(4, 0, x.data_ptr(), 0, y.data_ptr(), x.numel(), float(alpha), 0.0, stream_ptr())
        return y
    return _cpu.axpy(alpha, x, y)


def set_scalar(a: torch.Tensor, v: float) -> torch.Tensor:
    return a.fill_(v)


def zero(a: torch.Tensor) -> torch.Tensor:
    return a.zero_()


# ---- reductions (device scalar result)
def _reduce(op, a, b=None):
    if _gpu(a, b):
        out = torch.empty(1, dtype=torch.float32, device=a.device)
        ws = torch.empty(1024, dtype=torch.float32, device=a.device)
        kernels().reduce(op, a.data_ptr(), 0 if b is None else b.data_ptr(), a.numel(), ws.data_ptr(), out.data_ptr(),
                         stream_ptr())
        return out
    return _cpu.reduce(op, a, b)


def sum(a):  # noqa: A001
    return _reduce(0, a)


def dot_product(a, b):
    return _reduce(1, a, b)


def norm_squared(a):
    return _reduce(2, a)


def sum_squared_diff(a, b):
    return _reduce(3, a, b)


# ---- random fills (Philox-4x32-10 on the GPU)
def fill_random_uniform(a: torch.Tensor, low: float = 0.0, high: float = 1.0, seed: int = 0) -> torch.Tensor:
    if _gpu(a):
        kernels().fill_random(a.data_ptr(), a.numel(), int(seed) & ((1 << 64) - 1), float(low), float(high), 0,
                              stream_ptr())
        return a
    return _cpu.fill_random(a, low, high, seed, False)


def fill_random_normal(a: torch.Tensor, mean: float = 0.0, std: float = 1.0, seed: int = 0) -> torch.Tensor:
    if _gpu(a):
        kernels().fill_random(a.data_ptr(), a.numel(), int(seed) & ((1 << 64) - 1), float(mean), float(std), 1,
                              stream_ptr())
        return a
    return _cpu.fill_random(a, mean, std, seed, True)


# ---- layout
def transpose_2d(a: torch.Tensor, rows: int, cols: int, batch: int = 1) -> torch.Tensor:
    """[batch][rows][cols] -> [batch][cols][rows]."""
    if _gpu(a):
        out = torch.empty(batch * rows * cols, dtype=a.dtype, device=a.device)
        kernels().transpose_batched(a.data_ptr(), out.data_ptr(), batch, rows, cols, stream_ptr())
        return out.view(batch, cols, rows) if batch > 1 else out.view(cols, rows)
    return _cpu.transpose_2d(a, rows, cols, batch)


def nchw_to_cnhw(a: torch.Tensor) -> torch.Tensor:
    N, C, H, W = a.shape
    if _gpu(a):
        out = torch.empty((C, N, H, W), dtype=a.dtype, device=a.device)
        kernels().nchw_cnhw(a.data_ptr(), out.data_ptr(), N, C, H * W, 1, stream_ptr())
        return out
    return _cpu.swap01(a)


def cnhw_to_nchw(a: torch.Tensor) -> torch.Tensor:
    C, N, H, W = a.shape
    if _gpu(a):
        out = torch.empty((N, C, H, W), dtype=a.dtype, device=a.device)
        kernels().nchw_cnhw(a.data_ptr(), out.data_ptr(), N, C, H * W, 0, stream_ptr())
        return out
    return _cpu.swap01(a)
