"""Tensor ops (reference include/tensor/tensor_ops.hpp:14-255, CPU tensor_ops.hpp and CUDA
tensor_ops.cpp / tensor_kernels.cu): im2col / col2im, pad / unpad / crop, batch & channel
slicing, micro-batch split, channel softmax — NCHW, GPU tensors (fp32) on HIP kernels, CPU
tensors (fp32 / fp64) on the native C++ backend (``ops/cpu.py``)."""
from __future__ import annotations

from typing import List

import torch

from ..ops import cpu as _cpu
from ..ops._ext import kernels, stream_ptr


def _gpu(t: torch.Tensor) -> bool:
    if t.is_cuda:
        if t.dtype != torch.float32:
            raise TypeError("GPU tensor ops take float32 tensors")
        return True
    return False


def im2col(x: torch.Tensor, kh: int, kw: int, sh: int = 1, sw: int = 1, ph: int = 0, pw: int = 0) -> torch.Tensor:
    """col[(c, ky, kx)][n*OH*OW + oy*OW + ox] (reference column layout)."""
    if _gpu(x):
        from ..ops import hip
        return hip.im2col(x.contiguous(), kh, kw, sh, sw, ph, pw)
    return _cpu.im2col(x, kh, kw, sh, sw, ph, pw)


def col2im(col: torch.Tensor, x_shape, kh: int, kw: int, sh: int = 1, sw: int = 1, ph: int = 0, pw: int = 0):
    if _gpu(col):
        from ..ops import hip
        return hip.col2im(col, x_shape, kh, kw, sh, sw, ph, pw)
    return _cpu.col2im(col, x_shape, kh, kw, sh, sw, ph, pw)


def _pad_crop(x, OH, OW, top, left, value=0.0):
    N, C, H, W = x.shape
    out = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device)
    kernels().pad_crop(x.contiguous().data_ptr(), out.data_ptr(), N * C, H, W, OH, OW, top, left, float(value),
                       stream_ptr())
    return out


def pad(x: torch.Tensor, pad_h: int, pad_w: int, value: float = 0.0) -> torch.Tensor:
    """Pad H by pad_h and W by pad_w on both sides."""
    N, C, H, W = x.shape
    if _gpu(x):
        return _pad_crop(x, H + 2 * pad_h, W + 2 * pad_w, pad_h, pad_w, value)
    return _cpu.pad2d(x, pad_h, pad_w, value)


def unpad(x: torch.Tensor, pad_h: int, pad_w: int) -> torch.Tensor:
    N, C, H, W = x.shape
    if _gpu(x):
        return _pad_crop(x, H - 2 * pad_h, W - 2 * pad_w, -pad_h, -pad_w)
    return _cpu.crop2d(x, pad_h, pad_w, H - 2 * pad_h, W - 2 * pad_w)


def crop(x: torch.Tensor, start_h: int, start_w: int, end_h: int, end_w: int) -> torch.Tensor:
    """Rows start_h..end_h and columns start_w..end_w, inclusive (reference tensor_ops.hpp:564)."""
    N, C, H, W = x.shape
    if end_h >= H or end_w >= W or start_h > end_h or start_w > end_w:
        raise ValueError("Invalid crop dimensions")
    if _gpu(x):
        return _pad_crop(x, end_h - start_h + 1, end_w - start_w + 1, -start_h, -start_w)
    return _cpu.crop2d(x, start_h, start_w, end_h - start_h + 1, end_w - start_w + 1)


def slice_batch(x: torch.Tensor, start: int, end: int) -> torch.Tensor:
    if end > x.shape[0] or start > end:
        raise ValueError("Invalid batch slice range")
    return x[start:end].clone()


def slice_channels(x: torch.Tensor, start: int, end: int) -> torch.Tensor:
    if end > x.shape[1] or start > end:
        raise ValueError("Invalid channel slice range")
    return x[:, start:end].contiguous()


def split(x: torch.Tensor, num_splits: int) -> List[torch.Tensor]:
    """Split along the batch into ``num_splits`` parts; the last takes the remainder (micro-batching)."""
    n = x.shape[0]
    if num_splits <= 0 or num_splits > n:
        raise ValueError("Invalid number of splits")
    base = n // num_splits
    out, s = [], 0
    for i in range(num_splits):
        e = n if i == num_splits - 1 else s + base
        out.append(x[s:e].clone())
        s = e
    return out


def apply_softmax(x: torch.Tensor) -> torch.Tensor:
    """Softmax over the channel dimension at every (n, h, w) (in place; returns x)."""
    if _gpu(x):
        from ..ops import hip
        N, C, H, W = x.shape
        y = hip.softmax_channels(x.contiguous(memory_format=torch.channels_last))
        return x.copy_(y)
    return x.copy_(_cpu.softmax_channels(x))
