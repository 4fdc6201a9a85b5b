"""Flat parameter arena: one contiguous fp32 master buffer, one fp32 gradient buffer and (on the
GPU bf16 path) one bf16 shadow buffer for a whole model or pipeline stage.

Every layer parameter is a strided *view* into these buffers, so
  * the optimizer is ONE fused kernel over the flat buffer (reference: one launch per
    tensor, `include/nn/optimizers.hpp:147-156`),
  * gradient clearing is one memset, DP all-reduce buckets are plain slices,
  * conv weights use the channels_last view (logical {Cout,Cin,KH,KW} = the checkpoint shape,
    physical [Cout][KH][KW][Cin] = the MFMA B operand), so no repacking is ever needed.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

ALIGN = 64  # elements: keeps every view 256-byte aligned for float4 / 16-byte bf16x8 access


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    channels_last: bool = False


def _strides(shape, channels_last):
    if channels_last and len(shape) == 4:
        n, c, h, w = shape
        return (c * h * w, 1, w * c, c)
    st = []
    acc = 1
    for d in reversed(shape):
        st.append(acc)
        acc *= d
    return tuple(reversed(st))


class ParamArena:
    def __init__(self, specs: List[ParamSpec], device: torch.device, shadow_dtype: Optional[torch.dtype] = None,
                 dtype: torch.dtype = torch.float32):
        self.device = torch.device(device)
        self.dtype = dtype
        self.specs = list(specs)
        self.offsets = []
        off = 0
        for s in self.specs:
            self.offsets.append(off)
            n = 1
            for d in s.shape:
                n *= d
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = max(off, ALIGN)
        self.data = self.new_zeros(dtype)
        self.grad = self.new_zeros(dtype)
        self.shadow = self.new_zeros(shadow_dtype) if shadow_dtype is not None else None
        self._synced_version = -1
        self.step = 0  # optimizer steps applied (graph-replay safe counter lives in the optimizer)

    def new_zeros(self, dtype=None) -> torch.Tensor:
        """A zeroed flat buffer of the arena's size. On the GPU it comes from the native runtime's
        stream-ordered pool (device.py / csrc/kernels/runtime.cpp) — arenas, optimizer moments and
        their bf16 shadow are allocated once and live outside PyTorch's caching allocator."""
        dtype = dtype or self.dtype
        if self.device.type == "cuda":
            from ..device import get_device
            return get_device(self.device).allocate(self.numel, dtype, zero=True)
        return torch.zeros(self.numel, dtype=dtype, device=self.device)

    def _view(self, buf, i):
        s = self.specs[i]
        cl = s.channels_last and self.device.type == "cuda"
        return torch.as_strided(buf, s.shape, _strides(s.shape, cl), self.offsets[i])

    def param(self, i):
        return self._view(self.data, i)

    def grad_view(self, i):
        return self._view(self.grad, i)

    def shadow_view(self, i):
        return None if self.shadow is None else self._view(self.shadow, i)

    def zero_grad(self):
        if self.grad.is_cuda:
            from ..ops import hip
            hip.zero_(self.grad)  # the library's zero-fill kernel (no ATen fill in the step graph)
        else:
            self.grad.zero_()

    def sync_shadow(self, force: bool = False):
        """Refresh the bf16 shadow from the fp32 master if the master changed in place."""
        if self.shadow is None:
            return
        v = self.data._version
        if force or v != self._synced_version:
            if self.device.type == "cuda":
                from ..ops import hip
                hip.cast_bf16(self.data, self.shadow)
            else:
                self.shadow.copy_(self.data)
            self._synced_version = self.data._version

    def mark_synced(self):
        self._synced_version = self.data._version
